#!/bin/bash
# tools/mkvariant.sh NAME -- build the working tree's libpifft.so into
# abvar/NAME.so in a scratch copy (the in-tree build is left alone; abvar/ is
# git-ignored but travels to the GPU box); EXTRA="-D..." adds compile flags,
# KERNELS_H=file replaces csrc/pifft_kernels.h (e.g. an older revision).  The
# A/B timing of such variants is tools/ab.sh.
set -e
name="$1"
root="$(cd "$(dirname "$0")/.." && pwd)"
tmp="/tmp/pifft_variant_$name"
rm -rf "$tmp" && mkdir -p "$tmp/pkg" "$tmp/include"
cp -r "$root/cs87project-msolano2_amd/csrc" "$root/cs87project-msolano2_amd/Makefile" "$tmp/pkg/"
cp "$root/include/pifft.h" "$tmp/include/"
[ -n "${KERNELS_H:-}" ] && cp "$KERNELS_H" "$tmp/pkg/csrc/pifft_kernels.h"
make -s -j8 -C "$tmp/pkg" libpifft.so ROOT=.. EXTRA="${EXTRA:-}" > "$tmp/build.log" 2>&1
mkdir -p "$root/abvar"
cp "$tmp/pkg/libpifft.so" "$root/abvar/$name.so"
echo "abvar/$name.so"
