# round 6, session y: PMC traffic at HEAD of every config's plan and of one
# rank's plan of the 2/4/8-GPU split (FETCH_SIZE, WRITE_SIZE in separate
# rocprofv3 --pmc passes; tools/pmc_traffic.py) -> profiles/r06y_traffic_*.json,
# which the bench line's roofline.traffic / traffic_source read
set -o pipefail
bash tools/gpu_session.sh r06y p
