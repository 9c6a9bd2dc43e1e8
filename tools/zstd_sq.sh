#!/bin/bash
# SQ counters of rcdc_zstd_block_kernel on word text (tools/zstd_prof.py):
# two passes of at most 8 SQ counters each.  Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-zstd_sq}
KIND=${2:-text}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python -u tools/zstd_prof.py --gib 1 --reps 1 --kinds $KIND > $OUT/p$i.log 2>&1 || exit 1
done
echo done
