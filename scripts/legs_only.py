"""bench.py's config legs alone (no encode before them): isolates the legs' own timing."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from oracle import oracle  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.Stream()
for rep in range(2):
    legs = bench.config_legs(torch, dev, 0, st, oracle.OracleClay, 30)
    for k, v in legs.items():
        print(rep, k, v["kernel_ms_median"], v["kernel_ms_min"], v["path"], flush=True)
