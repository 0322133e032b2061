#!/bin/bash
# tools/isa_one.sh "<T>,<R>,<C>,<MODE>,<NTS>,<LP>" [extra hipcc flags]
# gfx950 assembly of ONE k_pass instantiation (device only) on stdout, for
# reading its LDS instructions, VGPR count and scratch (no GPU needed).
set -e
args="$1"; shift
d=$(mktemp -d)
cat > "$d/one.hip" <<EOT
#include "$(cd "$(dirname "$0")/.." && pwd)/cs87project-msolano2_amd/csrc/pifft_kernels.h"
template __global__ void pifft::k_pass<${args}>(pifft::PassArgs);
EOT
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off --cuda-device-only -S -o - "$@" "$d/one.hip"
rm -rf "$d"
