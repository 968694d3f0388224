"""Compat surface: `from utils import *`, vae-hpo CLI defaults, bench contract."""
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_utils_star_import_reexports():
    ns = {}
    exec("from utils import *", ns)
    for name in ("os", "socket", "psutil", "re", "torch", "dist", "init_comm_size_and_rank",
                 "get_comm_size_and_rank", "find_ifname", "parse_slurm_nodelist", "setup_ddp",
                 "setup_ddp_groups", "print0"):
        assert name in ns, name
    assert ns["get_comm_size_and_rank"]() == (1, 0)  # uninitialised -> (1, 0)


def _load_script(name):
    spec = importlib.util.spec_from_file_location(name.replace("-", "_"), os.path.join(ROOT, name))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_vae_hpo_cli_defaults():
    m = _load_script("vae-hpo.py")
    a = m.parse_args([])
    assert (a.batch_size, a.epochs, a.ngroups) == (128, 3, 2)


def test_bench_cpu_contract():
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--backend", "torch"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["n_gpus"] == 1 and out["steps"] == 3 and out["config"]["valid"]
    assert out["config"]["global_batch"] == 128


def test_native_extension_builds_and_loads():
    from multidisttorch_amd.ops import native

    C = native.ensure_built()
    assert C.ARCH == "gfx950"
    assert hasattr(C, "MlpVaeEngine") and hasattr(C, "BucketReducer")
