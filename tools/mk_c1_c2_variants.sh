#!/bin/bash
# tools/mk_c1_c2_variants.sh -- round 5: library variants for the round-4
# verdict's "two co-resident workgroups per CU" experiment on config 1: the
# working tree's libpifft.so plus fp64 1024-point strided passes at C = 2
# lines (128 threads: two workgroups per CU where C = 4 runs one), built
# plain (abvar2/c2x.so) and with the workgroup clocks (-DPIFFT_WG_CLOCK,
# abvar2/c2xclock.so; tools/wg_clock.py).  Select C = 2 with PIFFT_TUNING=1
# PIFFT_COL_C64=2 PIFFT_STRIDED_CMIN=2.
set -e
root="$(cd "$(dirname "$0")/.." && pwd)"
for v in c2x c2xclock; do
  tmp="/tmp/pifft_variant_$v"
  rm -rf "$tmp" && mkdir -p "$tmp/pkg" "$tmp/include"
  cp -r "$root/cs87project-msolano2_amd/csrc" "$root/cs87project-msolano2_amd/Makefile" "$tmp/pkg/"
  cp "$root/include/pifft.h" "$tmp/include/"
  for mode in 1 2; do echo "PK(double, 64, 1024, 2, $mode, 1, 0)," >> "$tmp/pkg/csrc/pifft_instances_0.inc"; done
  extra=""; [ "$v" = c2xclock ] && extra="-DPIFFT_WG_CLOCK"
  make -s -j8 -C "$tmp/pkg" libpifft.so ROOT=.. EXTRA="$extra" > "$tmp/build.log" 2>&1
  mkdir -p "$root/abvar2"
  cp "$tmp/pkg/libpifft.so" "$root/abvar2/$v.so"
  echo "abvar2/$v.so"
done
