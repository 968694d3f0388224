set -e
mkdir -p gpurun_out/r6_e2e
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 300 $R --master-port 29611 vae-hpo.py --ngroups 1 --model conv --synthetic --metrics-dir gpurun_out/r6_e2e/c28 > gpurun_out/r6_e2e/c28.log 2>&1
timeout -k 10 300 $R --master-port 29612 vae-hpo.py --ngroups 1 --model mlp --synthetic --metrics-dir gpurun_out/r6_e2e/mlp > gpurun_out/r6_e2e/mlp.log 2>&1
timeout -k 10 300 $R --master-port 29613 vae-hpo.py --ngroups 1 --model conv --image-size 128 --batch-size 64 --train-samples 8192 --test-samples 1024 --synthetic --metrics-dir gpurun_out/r6_e2e/c128 > gpurun_out/r6_e2e/c128.log 2>&1
grep -h MDT_AGGREGATE gpurun_out/r6_e2e/*.log
