# round 6, session z: the round's evidence at HEAD -- the GPU suite + smoke,
# bench.py as the driver runs it (the printed line + sidecar), and the
# rocprofv3 --kernel-trace --stats of the bench with tools/check_rooflines.py
set -o pipefail
bash tools/gpu_session.sh r06z tbs
