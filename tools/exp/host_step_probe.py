#!/usr/bin/env python3
"""host time of one SteppingDriver step of the fused C3 chain at the 1 MiB chunk,
doFilter (eager) vs doFilterGraphed (replay), via bench.host_step_costs; printed as JSON."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "cuda-sdr_amd"), REPO]

import torch  # noqa: E402

import bench  # noqa: E402
from gpusdr import ops  # noqa: E402

if __name__ == "__main__":
    for _ in range(3):
        print(json.dumps(bench.host_step_costs(ops, torch.device("cuda", 0), steps=200)), flush=True)
