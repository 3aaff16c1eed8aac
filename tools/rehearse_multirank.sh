mkdir -p gpurun_out
export MIVC_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --slots 32 --frames 16 > gpurun_out/rehearse2.log 2>&1
