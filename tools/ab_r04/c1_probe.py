"""The config-1 leg alone (bench.config1_leg on cuda:0): one JSON line."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from evolu_amd.engine import Engine  # noqa: E402

a = argparse.Namespace(steps=30, warmup=5, cpu_seconds=0)
eng = Engine(0)
print(json.dumps(bench.config1_leg(eng, a)))
eng.close()
