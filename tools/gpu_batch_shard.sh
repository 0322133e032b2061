set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "config3 or config1_2 or generator" > gpurun_out/batch_tests.log 2>&1 || { tail -20 gpurun_out/batch_tests.log; exit 1; }
tail -2 gpurun_out/batch_tests.log
timeout -k 10 120 python -u bench.py --log-n 12 --prec 32 --batch 4096 --shard batch --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/b_c3_1.log 2>&1 || exit 1
for g in 2 4 8; do timeout -k 10 120 python -u bench.py --log-n 12 --prec 32 --batch 4096 --shard batch --as-rank 0/$g --steps 50 --warmup 5 > gpurun_out/b_c3_as$g.log 2>&1 || exit 1; done
timeout -k 10 180 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --dist-backend gloo --same-device --log-n 12 --prec 32 --batch 4096 --shard batch --allgather --steps 5 --warmup 2 > gpurun_out/b_c3_gloo2.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py > gpurun_out/b_c4.log 2>&1 || exit 1
for f in b_c3_1 b_c3_as2 b_c3_as4 b_c3_as8 b_c3_gloo2 b_c4; do echo "== $f"; grep '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['n_gpus'], d['config']['workload'], d['config'].get('emulated_rank'), d['config']['allgather_ms'], d['roofline']['achieved'], d['roofline']['frac'])"; done
