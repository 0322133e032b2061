#!/bin/bash
# tools/gpu_r02f.sh -- HEAD evidence (tools/gpu_round2.sh r02f), then the
# hipGraph probe of the launch-bound configs (tools/probe_graph.py).
set -o pipefail
bash tools/gpu_round2.sh r02f || exit 1
timeout -k 10 180 python3 -u tools/probe_graph.py > gpurun_out/r02f/probe_graph.log 2>&1 || { cat gpurun_out/r02f/probe_graph.log; exit 1; }
cat gpurun_out/r02f/probe_graph.log
