"""Repeat tests/test_gpu_graph.py::test_bucketed_dp_plan_replay_bitwise under engine option overrides
(one process, sequential) and count failures: locating an intermittent plan-vs-eager mismatch.

usage: python tools/dp_race_probe.py REPS [KEY=VAL ...]"""
import os
import sys
import traceback

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-elasticity-predictor_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402
from alignn_mi355x import engine  # noqa: E402
import test_gpu_graph as T  # noqa: E402

reps = int(sys.argv[1])
over = dict(kv.split("=") for kv in sys.argv[2:])
orig = engine.AlignnEngine.__init__


def patched(self, cfg):
    orig(self, cfg)
    for k, v in over.items():
        setattr(self, k, type(getattr(self, k))(int(v)))


engine.AlignnEngine.__init__ = patched
fails = 0
for r in range(reps):
    try:
        T.test_bucketed_dp_plan_replay_bitwise()
    except AssertionError:
        fails += 1
        print("fail", r, traceback.format_exc().strip().splitlines()[-1], flush=True)
print(f"{over}: {fails}/{reps} failed", flush=True)
