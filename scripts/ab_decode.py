#!/usr/bin/env python3
"""A/B of planner options on the decode / repair configurations (device-resident, median
of RUNS).  Usage: CLAY_PLAN_MERGE=0|1 python scripts/ab_decode.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_paths as B  # noqa: E402

if __name__ == "__main__":
    B.prewarm(250)
    B.decode_cfg(4, 2, 5, 64 << 20, [0])
    B.decode_cfg(10, 4, 13, 1 << 30, [0, 4, 8, 12])
    B.decode_cfg(10, 4, 13, 1 << 30, [0])
    B.repair_cfg(9, 3, 11, 268_435_458, 0)
    B.encode_cfg(9, 3, 11, 9 * (256 << 20))
