#!/usr/bin/env python3
"""One parametrised driver for the GPU runs made through ``gpurun`` (it replaces
the one-off ``scripts/gpu_*.sh`` / ``run_*.sh`` of rounds 1-2; git history keeps
them, and every recipe they ran maps onto the steps below).

    python scripts/gpu_ab.py [--out gpurun_out/NAME] STEP [STEP ...]

STEP grammar. ``@K=V,K=V`` at the end of a step sets environment variables for
that step only (A/B switches such as MDT_CONV_F28=0, MDT_CONV_DIRECT=0):

  test[:PATH[:KEXPR]]                     pytest (default ``tests -m gpu``), one process
  testall[:PATH[:KEXPR]]                  the same without -x; plain test failures (exit 1) do not end the run
  bench[:MODEL[:B[:STEPS[:WARMUP]]]]      bench.py -> bench_<i>.json + a summary line
  driver[:ARG:ARG...]                     the driver's command: bench.py --gpus 1 --steps 20 --warmup 5 [ARGS]
  ddp:N[:MODEL[:B[:STEPS[:WARMUP]]]]      one trial of N replicas sharing the GPU (torchrun, gloo world,
                                          p2p data plane unless @MDT_REDUCER=... says otherwise)
  launches[:IMAGE[:B]]                    bench/conv_kernels.py (every launch of a step, alone)
  f28phases | f28parts | dconv[:B]        in-kernel stamp / per-launch tools of the fused kernels
  prof[:MODEL[:B]]                        rocprofv3 --kernel-trace --stats of a short bench run
  pmc:MODEL:B:CTR+CTR...                  one rocprofv3 --pmc pass (keep within the per-block limits)
  smoke                                   __graft_entry__.smoke()
  py:SCRIPT[:ARG...]                      python SCRIPT ARG... (diagnostics under bench/)

Every step runs under its own ``timeout -k 10``; the first failing step ends
the run with its exit status, so nothing else touches the GPU after a fault,
an abort or a time limit. This script never initialises the GPU itself: each
step is a child process.

Examples (on the box):
    python scripts/gpu_ab.py --out gpurun_out/ab test:tests/gpu/test_conv28_fused.py driver \\
        bench:conv28:128:200:20 bench:conv28:128:200:20@MDT_CONV_F28=0
    python scripts/gpu_ab.py pmc:conv128:64:SQ_INSTS_MFMA+SQ_VALU_MFMA_BUSY_CYCLES+SQ_BUSY_CYCLES
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable

LIMITS = {"test": 900, "testall": 900, "bench": 240, "ddp": 240, "driver": 180, "launches": 240, "f28phases": 120, "f28parts": 120,
          "dconv": 120, "prof": 300, "pmc": 90, "smoke": 300, "py": 300}


def parse(step):
    env = {}
    if "@" in step:
        step, kv = step.split("@", 1)
        for item in kv.split(","):
            k, v = item.split("=", 1)
            env[k] = v
    parts = step.split(":")
    return parts[0], parts[1:], env


def bench_args(model="conv28", b=None, steps="50", warmup="10"):
    a = [os.path.join(ROOT, "bench.py"), "--model", model, "--steps", steps, "--warmup", warmup]
    if b:
        a += ["--batch-size", b]
    return a


def command(kind, args, out, i):
    """(argv, cwd, stdout file, limit seconds) of one step."""
    log = os.path.join(out, f"{i:02d}_{kind}.log")
    if kind in ("test", "testall"):
        path = args[0] if args else "tests"
        argv = [PY, "-u", "-m", "pytest", path] + (["-x"] if kind == "test" else []) + [
            "-q", "-s", "--timeout", "150", "--timeout-method", "thread"]
        if not args:
            argv += ["-m", "gpu"]
        if len(args) > 1:
            argv += ["-k", args[1]]
        return argv, ROOT, log
    if kind == "bench":
        return [PY] + bench_args(*args), ROOT, os.path.join(out, f"{i:02d}_bench.json")
    if kind == "ddp":
        n = args[0]
        rest = bench_args(*(args[1:] or ["conv28"]))
        return [PY, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", n, "--master-addr",
                "127.0.0.1", "--master-port", str(29600 + i)] + rest + ["--gpus", n, "--ngroups", "1"], ROOT, \
            os.path.join(out, f"{i:02d}_ddp.json")
    if kind == "driver":
        return [PY, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "20", "--warmup", "5"] + args, ROOT, \
            os.path.join(out, f"{i:02d}_driver.json")
    if kind == "launches":
        image = args[0] if args else "128"
        b = args[1] if len(args) > 1 else "64"
        return [PY, os.path.join(ROOT, "bench", "conv_kernels.py"), "--image", image, "--batch", b, "--reps", "20",
                "--json", os.path.join(out, f"{i:02d}_launches.json")], ROOT, log
    if kind == "f28phases":
        return [PY, "-m", "multidisttorch_amd.obs.f28_phases", "--json", os.path.join(out, f"{i:02d}_phases.json")], \
            ROOT, log
    if kind == "f28parts":
        return [PY, os.path.join(ROOT, "bench", "f28_parts.py"), "--json",
                os.path.join(out, f"{i:02d}_parts.json")], ROOT, log
    if kind == "dconv":
        b = args[0] if args else "64"
        return [PY, os.path.join(ROOT, "bench", "dconv_stamps.py"), "--batch", b, "--json",
                os.path.join(out, f"{i:02d}_dconv.json")], ROOT, log
    if kind == "prof":
        model = args[0] if args else "conv28"
        b = args[1] if len(args) > 1 else None
        d = os.path.join(out, f"{i:02d}_prof")
        return ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", d, "-o", "prof", "--",
                PY] + bench_args(model, b, "20", "5"), "/tmp", log
    if kind == "pmc":
        model, b, ctrs = args[0], args[1], args[2].split("+")
        d = os.path.join(out, f"{i:02d}_pmc")
        return ["rocprofv3", "--pmc"] + ctrs + ["--kernel-trace", "--output-format", "csv", "-d", d, "-o", "pmc",
                                               "--", PY] + bench_args(model, b, "6", "2") + ["--no-graphs"], "/tmp", log
    if kind == "py":
        return [PY, os.path.join(ROOT, args[0])] + args[1:], ROOT, log
    if kind == "smoke":
        return [PY, "-c", "import __graft_entry__ as g; g.smoke(); print('smoke ok')"], ROOT, log
    raise SystemExit(f"unknown step kind {kind!r}")


def summary(kind, path):
    if kind in ("bench", "driver", "ddp"):
        try:
            with open(path) as f:
                line = [l for l in f if l.startswith("{")][-1]
            d = json.loads(line)
            c = d["config"]
            extra = f" {c['parallelism']} {c.get('reducer')} equal={c.get('replicas_bitwise_equal')}" \
                if kind == "ddp" else ""
            return f"{c['model']} B={c['global_batch']}: {d['ms_per_step']} ms/step, {d['value']:.0f} {d['unit']}{extra}"
        except Exception as e:  # noqa: BLE001 - report, do not crash the run
            return f"(no JSON line: {e})"
    with open(path, errors="replace") as f:
        lines = [l.rstrip() for l in f if "amdgpu.ids" not in l]
    return "\n".join(lines[-12:])


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "ab"))
    ap.add_argument("steps", nargs="+")
    a = ap.parse_args()
    a.out = os.path.abspath(a.out)
    os.makedirs(a.out, exist_ok=True)
    for i, step in enumerate(a.steps):
        kind, args, env_add = parse(step)
        argv, cwd, out = command(kind, args, a.out, i)
        limit = LIMITS[kind]
        if kind == "pmc":  # a pass over-subscribing a counter block hangs: hard kill
            full = ["timeout", "-s", "KILL", str(limit)] + argv
        else:
            full = ["timeout", "-k", "10", str(limit)] + argv
        env = dict(os.environ, **env_add)
        if kind == "ddp":  # ranks share the GPU: RCCL refuses that, so a gloo world + the p2p data plane
            env.setdefault("DDP_BACKEND", "gloo")
            env.setdefault("MDT_REDUCER", "p2p")
        if kind in ("prof", "pmc"):
            env["TMPDIR"] = "/tmp"
        print(f"== [{i}] {step}", flush=True)
        json_out = kind in ("bench", "driver", "ddp")  # stdout is the JSON line; stderr apart
        with open(out, "w") as f, open(out + ".err" if json_out else os.devnull, "w") as fe:
            r = subprocess.run(full, cwd=cwd, env=env, stdout=f, stderr=fe if json_out else subprocess.STDOUT)
        print(summary(kind, out), flush=True)
        if r.returncode != 0 and json_out:
            print(summary("log", out + ".err"), flush=True)
        if r.returncode == 1 and kind == "testall":
            print(f"== step {i} ({step}): test failures (see {out}); continuing", flush=True)
            continue
        if r.returncode != 0:
            print(f"== step {i} ({step}) failed with status {r.returncode}; stopping", flush=True)
            sys.exit(r.returncode)
    print("== all steps passed")


if __name__ == "__main__":
    main()
