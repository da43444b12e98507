#!/usr/bin/env python3
"""bench.py's input-path extra alone (host vs GPU inflate of site files, one
block and a stream of blocks), for a few block sizes.  One JSON line each.
    python tools/bench_input_path.py [--blocks 64,128,256]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", default="128")
    a = ap.parse_args()
    import torch

    import bench
    dev = torch.device("cuda", 0)
    for b in [int(x) for x in a.blocks.split(",")]:
        print(json.dumps({"block": b, **bench.bench_input_path(2160, 2560, dev, block=b)}), flush=True)


if __name__ == "__main__":
    main()
