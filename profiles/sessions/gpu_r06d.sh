# round 6, session d: on the pruned library (845 instances) -- the whole GPU
# suite + smoke, recording the instances again (the list must not grow); the
# A/B of MODE 11's tree-twiddle fetch against HEAD's kernels (abvar/base.so);
# config 2's workgroup chain; config 2 with 4-line second-pass tiles
# (PIFFT_WIL_CMIN=4: 256 workgroups instead of 128); one rank's plan of the
# G-GPU split for G = 1, 2, 4, 8 (--as-rank 0/G, the per-GPU time of the
# driver's scaling curve)
set -o pipefail
out=gpurun_out/r06d
mkdir -p $out
export PIFFTTEST_RECORD_INSTANCES=$out/instances_tests.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > $out/gpu_tests.txt 2>&1 && \
unset PIFFTTEST_RECORD_INSTANCES && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 && \
for shape in "--log-n 20 --workers 8" "--log-n 19 --workers 8" "--log-n 20 --workers 4" "--log-n 18 --workers 4" "--log-n 22 --workers 8" "--log-n 16 --workers 16"; do
  AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh "$shape --steps 400 --warmup 100" abvar/base.so cs87project-msolano2_amd/libpifft.so >> $out/ab_tree_fetch.txt 2>&1 || exit 1
done && \
timeout -k 10 120 python -u tools/wg_clock.py --log-n 20 --workers 8 > $out/wgc_c2.txt 2>&1 && \
timeout -k 10 120 python -u tools/tune.py --log-n 20 --workers 8 --steps 1000 --warmup 250 --check --variants '[{}, {"PIFFT_WIL_CMIN": "4"}, {}, {"PIFFT_WIL_CMIN": "4"}]' > $out/c2_wil_cmin4.txt 2>&1 && \
for g in 1 2 4 8; do
  timeout -k 10 200 python -u bench.py --as-rank 0/$g --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --detail $out/rank0of${g}_detail.json > $out/rank0of$g.txt 2>&1 || exit 1
done
