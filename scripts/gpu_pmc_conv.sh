# PMC counters per conv kernel, register-staged vs LDS-DMA path
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmcc/avail.txt 2>&1 || true
for impl in 1 0; do
  export MDT_CONV_GLDS=$impl
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-trace --output-format csv -d $R/gpurun_out/pmcc/a$impl -- python3 $R/bench/conv_kernels.py --reps 2 > $R/gpurun_out/pmcc/a$impl.log 2>&1 || exit $?
  timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $R/gpurun_out/pmcc/b$impl -- python3 $R/bench/conv_kernels.py --reps 2 > $R/gpurun_out/pmcc/b$impl.log 2>&1 || exit $?
  timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmcc/c$impl -- python3 $R/bench/conv_kernels.py --reps 2 > $R/gpurun_out/pmcc/c$impl.log 2>&1 || exit $?
done
