# Fused 28x28 step iteration: numerics tests, per-phase timing, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${MDT_OUT:-f28i}
mkdir -p $O
export MASTER_ADDR=127.0.0.1
timeout -k 10 300 python -u -m pytest tests/gpu/test_conv28_fused.py -x -q --timeout 120 --timeout-method thread > $O/pytest_f28.log 2>&1 || { tail -40 $O/pytest_f28.log; exit 1; }
tail -1 $O/pytest_f28.log
timeout -k 10 120 python -m multidisttorch_amd.obs.f28_phases --json $O/phases.json > $O/phases.txt 2>&1 || { tail -30 $O/phases.txt; exit 1; }
grep -v amdgpu.ids $O/phases.txt
timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 > $O/bench_200_20.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
python -c "import json;d=json.load(open('$O/bench_200_20.json'));print('bench', d['ms_per_step'], 'ms/step', d['value'])"
if [ "${PMC:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc1 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-graphs > $GRAFT_REPO_ROOT/$O/pmc1.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/pmc1.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc2 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-graphs > $GRAFT_REPO_ROOT/$O/pmc2.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/pmc2.log; }
  echo pmc done
fi
