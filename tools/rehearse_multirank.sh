cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HPCJOIN_SHARE_GPU=1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --inner 1e8 --outer 1e8 --steps 3 --warmup 1 > gpurun_out/rehearse2.log 2>&1; rc=$?
tail -5 gpurun_out/rehearse2.log; exit $rc
