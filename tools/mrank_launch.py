#!/usr/bin/env python3
"""Start N ranks of a program on this node, each optionally under its own
rocprofv3 kernel trace -- what torch.distributed.run does for bench.py, but
with the profiler wrapping each rank's own process (rocprofv3 must sit
directly in front of the program it profiles; it cannot wrap the launcher).
This process never touches the GPU.

    python tools/mrank_launch.py --np 2 --prof gpurun_out/trace2 -- bench.py --gpus 2 --grid 24 ...

Each rank gets RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1 and one
MASTER_PORT; rank r's trace goes to <prof>/r<r>.  Exits with the first
non-zero rank status (or 0)."""
import argparse
import os
import random
import subprocess
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--np", type=int, default=2)
    ap.add_argument("--prof", default=None, help="directory for the per-rank rocprofv3 kernel traces")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    assert cmd, "no program given"
    port = str(29100 + random.randrange(800))
    procs = []
    for r in range(a.np):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.np), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, LOCAL_WORLD_SIZE=str(a.np))
        argv = ["python3"] + cmd
        if a.prof:
            argv = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", os.path.join(a.prof, "r%d" % r),
                    "-o", "run", "--"] + argv
        procs.append(subprocess.Popen(argv, env=env))
    codes = [p.wait() for p in procs]
    print("rank exit codes:", codes, flush=True)
    sys.exit(next((c for c in codes if c), 0))


if __name__ == "__main__":
    main()
