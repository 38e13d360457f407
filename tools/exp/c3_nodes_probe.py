#!/usr/bin/env python3
"""bench.py's C3 node-path leg on its own (fused and unfused SteppingDriver
steps), printed as JSON; run under rocprofv3 --kernel-trace to see which launches a step makes."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "cuda-sdr_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
from gpusdr import ops  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    print(json.dumps(bench.node_path(ops, dev, 1.0, segments=int(os.environ.get("SEGMENTS", "11")))), flush=True)
