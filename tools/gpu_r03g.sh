#!/bin/bash
# tools/gpu_r03g.sh -- the rest of the GPU suite after a failure at a known
# test (resume from that file), then bench.py and the rocprofv3 roofline check
set -o pipefail
bash tools/gpu_r03.sh r03g "tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_fullsize.py"
