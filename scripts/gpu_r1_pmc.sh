# Round-1 checkpoint on one MI355X: GPU tests, bench (3 models), kernel-trace stats,
# and per-kernel PMC passes (MFMA busy / bf16 MOPs, LDS instrs + bank conflicts,
# HBM fetch / write bytes) on the eager (non-graph) conv28 and conv128 steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1pmc
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
timeout -k 10 180 python3 bench.py > $O/bench_conv28.json 2> $O/bench_conv28.err || { tail $O/bench_conv28.err; exit 1; }
timeout -k 10 180 python3 bench.py --model conv128 --batch-size 64 > $O/bench_conv128.json 2> $O/bench_conv128.err || exit 1
timeout -k 10 180 python3 bench.py --model mlp > $O/bench_mlp.json 2> $O/bench_mlp.err || exit 1
cat $O/bench_*.json
cd /tmp
timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2>&1 || true
for m in conv28 conv128; do
  bs=128; [ $m = conv128 ] && bs=64
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$m -o run -- python3 $R/bench.py --model $m --batch-size $bs --steps 200 --warmup 20 > $O/stats_$m.log 2>&1 || { tail -20 $O/stats_$m.log; exit 1; }
done
want() { for c in "$@"; do grep -qw "$c" $O/avail.txt && printf '%s ' "$c"; done; }
PA=$(want SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE)
PB=$(want SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR)
PC=$(want FETCH_SIZE GRBM_GUI_ACTIVE)
PD=$(want WRITE_SIZE)
echo "PA=$PA"; echo "PB=$PB"; echo "PC=$PC"; echo "PD=$PD"
for m in conv28 conv128; do
  bs=128; [ $m = conv128 ] && bs=64
  i=0
  for P in "$PA" "$PB" "$PC" "$PD"; do
    i=$((i+1))
    [ -z "$P" ] && continue
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/pmc_${m}_$i -- python3 $R/bench.py --model $m --batch-size $bs --steps 6 --warmup 2 --no-graphs > $O/pmc_${m}_$i.log 2>&1 || { tail -20 $O/pmc_${m}_$i.log; exit 1; }
  done
done
echo done
