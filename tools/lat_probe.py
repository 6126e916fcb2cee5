"""Burst latency probe: bench.py's plugin_bursts alone (tools/, not product)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from mtcp_amd import gpucsum  # noqa: E402

torch.cuda.init()
print(json.dumps(bench.plugin_bursts(gpucsum)))
