"""The one-GPU rehearsal tool MDT_CU_SPLIT (runtime/env.py::apply_cu_split):
HSA_CU_MASK set before HIP initialises confines a process's kernels to its
share of the CUs (checked with a probe grid that records where each
workgroup ran)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(HERE, "cu_mask_probe.py")], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1][7:])


def test_cu_split_confines_a_rank_to_its_share():
    full = _run({"MDT_CU_SPLIT": "0"})
    half = _run({"MDT_CU_SPLIT": "1", "LOCAL_RANK": "1", "LOCAL_WORLD_SIZE": "2"})
    quarter = _run({"MDT_CU_SPLIT": "1", "LOCAL_RANK": "0", "LOCAL_WORLD_SIZE": "4"})
    print(full, half, quarter)
    assert full["mask"] is None and full["distinct_cus"] > 200
    assert half["mask"] == "0:128-255" and half["distinct_cus"] <= 128
    assert quarter["mask"] == "0:0-63" and quarter["distinct_cus"] <= 64
