# round 6, session c: the whole GPU suite at the working tree (MODE 11's tree
# twiddles fetched in one round trip, tree_tw_fetch) recording every instance
# the tests' plans launch or the planner finds (tests/golden/instances_tests.txt);
# the A/B of the fetch against HEAD's kernels (abvar/base.so) on config 2 and
# neighbours; config 2's workgroup chain again
set -o pipefail
mkdir -p gpurun_out/r06c
export PIFFTTEST_RECORD_INSTANCES=gpurun_out/r06c/instances_tests.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/r06c/gpu_tests.txt 2>&1 && \
unset PIFFTTEST_RECORD_INSTANCES && \
for shape in "--log-n 20 --workers 8" "--log-n 19 --workers 8" "--log-n 20 --workers 4" "--log-n 18 --workers 4" "--log-n 22 --workers 8" "--log-n 16 --workers 16"; do
  AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh "$shape --steps 400 --warmup 100" abvar/base.so cs87project-msolano2_amd/libpifft.so >> gpurun_out/r06c/ab_tree_fetch.txt 2>&1 || exit 1
done && \
timeout -k 10 120 python -u tools/wg_clock.py --log-n 20 --workers 8 > gpurun_out/r06c/wgc_c2.txt 2>&1
