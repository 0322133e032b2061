# round 6, session e: every C4 pass against a copy with its own maps
# (tools/probe_c4_passes.hip, fp64 and fp32); config 2 with both passes on
# 256 CUs (fused pass at J = 2 / 4096-value tile -> radices 256.512, vs the
# default 128.1024 whose second pass has 128 workgroups), its neighbours; C1
# with plain (non-temporal off) streaming
set -o pipefail
out=gpurun_out/r06e
mkdir -p $out
timeout -k 10 200 ./tools/probe_c4_passes_bin 3 > $out/c4_pass_ceilings.log 2>&1 && \
for shape in "--log-n 20 --workers 8" "--log-n 19 --workers 8" "--log-n 21 --workers 8"; do
  PIFFT_LIB=abvar/j2full.so timeout -k 10 200 python -u tools/tune.py $shape --steps 1000 --warmup 250 --check \
    --variants '[{}, {"PIFFT_WIL_FUSE_J": "2", "PIFFT_WIL_FUSE_TILE": "4096"}, {}, {"PIFFT_WIL_FUSE_J": "2", "PIFFT_WIL_FUSE_TILE": "4096"}]' >> $out/c2_j2.txt 2>&1 || exit 1
done && \
timeout -k 10 200 python -u tools/tune.py --log-n 20 --workers 1 --steps 1000 --warmup 250 --check \
    --variants '[{}, {"PIFFT_NT": "0"}, {}, {"PIFFT_NT": "0"}]' > $out/c1_nt.txt 2>&1
