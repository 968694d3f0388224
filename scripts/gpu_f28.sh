# Fused 28x28 step: numerics tests first (one process, bounded), then the
# driver's bench command, the layer-path A/B and a kernel-stats profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${MDT_OUT:-f28}
mkdir -p $O
export MASTER_ADDR=127.0.0.1
timeout -k 10 300 python -u -m pytest tests/gpu/test_conv28_fused.py -x -v -s --timeout 120 --timeout-method thread > $O/pytest_f28.log 2>&1 || { tail -60 $O/pytest_f28.log; exit 1; }
grep -E "PASS|FAIL|rel-err" $O/pytest_f28.log | tail -12
for r in 1 2; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd_$r.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
  cat $O/driver_cmd_$r.json
done
timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 > $O/bench_200_20.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/bench_200_20.json
MDT_CONV_F28=0 timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 > $O/bench_layerpath.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/bench_layerpath.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o conv28 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
