#!/bin/bash
# tools/mkvariant.sh NAME -- build the working tree's libpifft.so into
# variants/NAME.so in a scratch copy (the in-tree build is left alone); the
# A/B timing of such variants is tools/ab.sh.
set -e
name="$1"
root="$(cd "$(dirname "$0")/.." && pwd)"
tmp="/tmp/pifft_variant_$name"
rm -rf "$tmp" && mkdir -p "$tmp/pkg" "$tmp/include"
cp -r "$root/cs87project-msolano2_amd/csrc" "$root/cs87project-msolano2_amd/Makefile" "$tmp/pkg/"
cp "$root/include/pifft.h" "$tmp/include/"
make -s -j8 -C "$tmp/pkg" libpifft.so ROOT=.. EXTRA="${EXTRA:-}" > "$tmp/build.log" 2>&1
mkdir -p "$root/variants"
cp "$tmp/pkg/libpifft.so" "$root/variants/$name.so"
echo "variants/$name.so"
