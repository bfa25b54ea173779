#!/usr/bin/env python3
"""cProfile of one bench.py run (host side): where the per-step issue time goes, and
which calls block on the GPU.  Arguments are bench.py's.

    RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29551 \\
        python tools/prof_bench.py --force-shard --workload hier_fedbuff --steps 5 --warmup 2
"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import bench
    sys.argv = ["bench.py"] + sys.argv[1:]
    pr = cProfile.Profile()
    pr.enable()
    bench.main()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(40)
