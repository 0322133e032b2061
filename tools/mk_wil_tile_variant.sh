#!/bin/bash
# tools/mk_wil_tile_variant.sh -- round 5: a library variant for the fused
# all-worker tree pass (MODE 11) at a 4096-value tile: the working tree's
# libpifft.so plus MODE 11 instances at smaller tiles (list below; P = 2..16)
# -> abvar2/wiltile.so.  Config 2's fused pass
# at the 8192-value tile has 128 workgroups on 256 CUs; at 4096 it has 256.
# Select with PIFFT_TUNING=1 PIFFT_WIL_FUSE_TILE=4096 [PIFFT_WIL_FUSE_J=4|8]
# [PIFFT_WIL_FUSE_VPT=8] [PIFFT_WIL_CMIN=4].
set -e
root="$(cd "$(dirname "$0")/.." && pwd)"
v=wiltile
tmp="/tmp/pifft_variant_$v"
rm -rf "$tmp" && mkdir -p "$tmp/pkg" "$tmp/include"
cp -r "$root/cs87project-msolano2_amd/csrc" "$root/cs87project-msolano2_amd/Makefile" "$tmp/pkg/"
cp "$root/include/pifft.h" "$tmp/include/"
# (T prec tile J) beside the default 8192-value tile's J = 16 / 8 / 4 (fp64)
# and 32 / 16 / 8 (fp32): fp64 4096 (J = 2, 4, 8), 2048 (J = 2, 4), 8192
# (J = 2); fp32 8192 (J = 2, 4), 4096 (J = 2, 4)
k=0
for spec in "double 64 4096 2" "double 64 4096 4" "double 64 4096 8" "double 64 2048 2" "double 64 2048 4" \
            "double 64 8192 2" "float 32 8192 2" "float 32 8192 4" "float 32 4096 2" "float 32 4096 4"; do
  set -- $spec
  for lp in 1 2 3 4; do
    C=$(($4 << lp)); R=$(($3 / C))
    [ $R -lt 16 ] && continue
    for nts in 0 1; do
      echo "PK($1, $2, $R, $C, 11, $nts, $lp)," >> "$tmp/pkg/csrc/pifft_instances_$((k % 8)).inc"
      k=$((k + 1))
      [ "$1" = double ] && [ $3 = 4096 ] && [ $4 = 4 ] && [ $lp -le 3 ] && echo "PKV($1, $2, $R, $C, 11, $nts, $lp, 8)," >> "$tmp/pkg/csrc/pifft_instances_$((k % 8)).inc"
    done
  done
done
make -s -j8 -C "$tmp/pkg" libpifft.so ROOT=.. > "$tmp/build.log" 2>&1 || { tail -30 "$tmp/build.log"; exit 1; }
mkdir -p "$root/abvar2"
cp "$tmp/pkg/libpifft.so" "$root/abvar2/$v.so"
echo "abvar2/$v.so"
