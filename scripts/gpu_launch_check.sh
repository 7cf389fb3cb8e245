# GPU: the driver's torchrun launch of bench.py at N=1, then every bench_configs line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 2 \
  --no-cpu-baseline > $O/bench_torchrun.log 2>&1 || exit $?
tail -1 $O/bench_torchrun.log
timeout -k 10 700 python -u bench_configs.py > $O/configs.jsonl 2> $O/configs.err || exit $?
cat $O/configs.jsonl
