"""The multi-rank bench launcher on the device (the path the driver's
8-GPU run takes): `bench.py --gpus 2` re-launches itself under
torch.distributed.run as a child process before touching the GPU
(bench.py spawn_ranks), each rank chunks its own streams (per-file
sharding, archiver.rs:195) and rank 0 prints one JSON line.  On a one-GPU
box the ranks share cuda:0 and time over gloo (RCDC_BENCH_BACKEND=gloo)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo(gpu_ctx):
    env = dict(os.environ, RCDC_BENCH_BACKEND="gloo")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--workload", "C2", "--steps", "2", "--warmup", "1", "--prewarm", "0",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=300,
                       env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert line["parity"]["mismatches"] == 0
    assert line["parity"]["streams_checked"] == 1024
    assert line["value"] > 0 and line["scaling"] == "weak"


def _two_ranks(args, n=2):
    env = dict(os.environ, RCDC_BENCH_BACKEND="gloo")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n)] + args +
                       ["--warmup", "1", "--prewarm", "0", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == n and line["value"] > 0
    return line


def test_bench_two_ranks_c4(gpu_ctx):
    """C4 over two ranks: LPT shares of 256 files (~7.5
    GiB per rank: walked), one resident batch per rank, pipelined passes, the
    parity counts of the 64-file sample summed over the ranks (all_reduce) --
    the path of the driver's 8-GPU C4 run."""
    line = _two_ranks(["--workload", "C4", "--c4-files", "256", "--steps", "2"])
    assert line["parity"]["files_checked"] == 256  # every file of both shares
    assert line["parity"]["mismatches"] == 0
    assert line["roofline"]["pipelined"] is True


def test_bench_two_ranks_c5(gpu_ctx):
    """C5 over two ranks: one 512 MiB zero stream sliced with max + 64 halos,
    the cross-rank stitch (shard.SlicedStream: the crossing window of each
    rank's device cut list, rcdc_plan_window, in one fixed-size all_gather)
    inside every timed step; rank 0's cuts against the closed form and the
    oracle."""
    line = _two_ranks(["--workload", "C5", "--stream-bytes", str(256 << 20), "--steps", "2"])
    assert line["parity"]["mismatches"] == 0
    assert line["parity"]["cuts"] >= (256 << 20) // (512 << 10) - 1
    assert line["config"]["stream_bytes_total"] == 512 << 20


# ---- the driver's 8-GPU run, rehearsed: 8 ranks on the one GPU over gloo
def test_bench_eight_ranks_c3(gpu_ctx):
    """C3 at 8 ranks (4 x 64 MiB streams each): every rank's walk, the
    timing barrier and max over 8 ranks, rank 0's parity over its streams."""
    line = _two_ranks(["--streams", "4", "--stream-bytes", str(64 << 20), "--steps", "2",
                       "--no-ingest"], n=8)
    assert line["parity"]["mismatches"] == 0 and line["parity"]["streams_checked"] == 4


def test_bench_eight_ranks_c4(gpu_ctx):
    """C4 at 8 ranks: LPT shares of 64 files, the sampled parity summed over
    the ranks."""
    line = _two_ranks(["--workload", "C4", "--c4-files", "64", "--steps", "2"], n=8)
    assert line["parity"]["mismatches"] == 0
    assert line["parity"]["files_checked"] == 64


def test_bench_eight_ranks_c5(gpu_ctx):
    """C5 at 8 ranks: one 512 MiB zero stream (64 MiB per rank), the stitch
    over fixed-size crossing windows in every timed step."""
    line = _two_ranks(["--workload", "C5", "--stream-bytes", str(64 << 20), "--steps", "2"],
                      n=8)
    assert line["parity"]["mismatches"] == 0
    assert line["config"]["stream_bytes_total"] == 512 << 20
    # the per-step stitch (plan end -> window, all_gather, .cpu(), host walk)
    assert line["stitch"]["ms_per_step_max_rank"] > 0 and line["stitch"]["backend"] == "gloo"
