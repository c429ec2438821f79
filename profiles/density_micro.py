"""Runs only bench.py's density microbench (16.7M-particle
lattice, one pure density pass from a fresh hash) and prints its JSON;
used for kernel A/B runs and rocprofv3 --pmc passes.

    python profiles/density_micro.py [--side 4096] [--reps 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    lpe = bench._load("lpe", os.path.join(bench.PKG, "lpe.py"))
    scenes = bench._load("scenes", os.path.join(bench.PKG, "scenes.py"))
    print(json.dumps(bench.density_microbench(lpe, scenes, 0, side=a.side, reps=a.reps)), flush=True)


if __name__ == "__main__":
    main()
