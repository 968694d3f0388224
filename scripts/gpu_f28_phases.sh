# Fused 28x28 step: per-phase in-kernel timing + kernel stats + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${MDT_OUT:-f28p}
mkdir -p $O
export MASTER_ADDR=127.0.0.1
timeout -k 10 120 python -m multidisttorch_amd.obs.f28_phases --json $O/phases.json > $O/phases.txt 2>&1 || { tail -30 $O/phases.txt; exit 1; }
cat $O/phases.txt
timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 > $O/bench_200_20.json 2>$O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/bench_200_20.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o conv28 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/kstats.py $O/prof/conv28_kernel_trace.csv | head -8
