"""Run bench.next_rows() alone (f3/f4 measurements) and print its JSON."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

torch.cuda.set_device(0)
print(json.dumps(bench.next_rows(torch.device("cuda", 0))))
