"""Failure isolation of the default intra-group data plane (the fused xGMI
all-reduce jobs, comm_jobs.h) -- the counterpart of the process-group
timeout / watchdog the reference relies on (/root/reference/utils.py:139,
SURVEY.md section 5).

Two ranks of one conv-VAE trial share the box's GPU (gloo world, CU-split, the
xgmi reducer forced as on an intra-node RCCL group). Rank 1 stops issuing
steps mid-epoch (``MDT_FAULT=rank=1,step=...``) while rank 0 has the whole
epoch enqueued, so every later step of rank 0 waits in-kernel for pushes that
never come. The survivor must notice through the trial watch, abort its
reducer (host-mapped abort word), drain its stream in seconds -- not one
``MDT_P2P_TIMEOUT_S`` (60 s here) per queued wait -- fail the trial with
TrialTimeout and still reach the final gloo barrier.
"""
import json
import os
import re
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def test_fused_xgmi_peer_loss_drains_fast_and_fails_trial():
    from multidisttorch_amd.launch import launch

    env = {"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2", "DDP_BACKEND": "gloo", "MDT_REDUCER": "xgmi",
           "MDT_CU_SPLIT": "1", "MDT_FAULT": "rank=1,step=12", "MDT_P2P_TIMEOUT_S": "60",
           "MDT_HEARTBEAT_S": "5", "MDT_ABORT_DRAIN_S": "30"}
    cmd = [sys.executable, os.path.join(ROOT, "vae-hpo.py"), "--model", "conv", "--ngroups", "1", "--epochs", "1",
           "--no-epoch-offset", "--synthetic", "--train-samples", str(128 * 60), "--test-samples", "256",
           "--no-results", "--graph-steps", "10"]
    rc, outs = launch(cmd, 2, emulate="torchrun", timeout=110, extra_env=env, capture=True)
    text0, text1 = outs[0] or "", outs[1] or ""
    assert rc == 0, (text0[-3000:], text1[-3000:])
    # the faulting rank failed its trial on purpose; the survivor noticed and aborted
    assert "InjectedFault" in text1, text1[-3000:]
    m = re.search(r"FAILED: TrialTimeout: .*\(stream drained in ([0-9.]+) s\)", text0)
    assert m, text0[-3000:]
    assert float(m.group(1)) <= 5.0, m.group(0)
    # both ranks reached the final global (gloo) barrier and reported
    assert re.search(r"^0 Done\. time: ", text0, re.M) and re.search(r"^1 Done\. time: ", text1, re.M)
    agg = [json.loads(l[len("MDT_AGGREGATE "):]) for l in text0.splitlines() if l.startswith("MDT_AGGREGATE ")]
    assert agg and agg[0]["failed_trials"] == [0], agg
