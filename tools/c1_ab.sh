# C1 pass breakdown A/B (tools/c1_profile.py): the pipe on / off, and the
# host-path phase timing of the stream passes (RCDC_HOST_PROFILE=1).
set -o pipefail
for a in 1 0 1 0; do
  RCDC_READ_AHEAD=$a timeout -k 10 120 python tools/c1_profile.py 256 10 | sed "s/^/pipe $a: /" || exit 1
done
RCDC_HOST_PROFILE=1 timeout -k 10 120 python tools/c1_profile.py 256 10 2>&1 | grep -v amdgpu.ids || exit 1
