# rocprofv3 kernel trace of the default bench (pipelined C3), kept for analysis
set -o pipefail
OUT=gpurun_out/${1:-tr}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u bench.py --steps 10 --warmup 3 --prewarm 0.2 --no-cpu-baseline --no-parity $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err || exit 1
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python - "$f" > $OUT/summary.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if 'rcdc' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
t0 = int(rows[0]['Start_Timestamp'])
for r in rows[-60:]:
    s, e = int(r['Start_Timestamp']) - t0, int(r['End_Timestamp']) - t0
    print(f"{r['Kernel_Name'][:40]:40s} q{r.get('Queue_Id','?')} {s/1e3:10.1f} {e/1e3:10.1f} {(e-s)/1e3:8.1f} grid {r.get('Grid_Size','?')}")
PY
cp $f $OUT/trace.csv
tail -40 $OUT/summary.txt
