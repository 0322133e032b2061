set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c1
timeout -k 10 300 python -u bench.py --gpus 8 --same-device --dist-backend gloo --log-n 22 --c5-log-n 24 --steps 3 --warmup 1 > gpurun_out/c1/rehearse8.log 2>&1 || { tail -30 gpurun_out/c1/rehearse8.log; exit 1; }
grep '^{' gpurun_out/c1/rehearse8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['config']['allgather_ms'], json.dumps(d['config']['secondary'])[:400]); print([ (r['rank'], r['ms_per_step']) for r in d['config']['per_rank']])"
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/c1/pmc -o pmc -- python3 -u tools/tune.py --log-n 20 --prec 64 --steps 5 --warmup 2 > gpurun_out/c1/pmc.out 2>&1 || { tail gpurun_out/c1/pmc.out; exit 1; }
C2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR"
timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d gpurun_out/c1/pmc2 -o pmc -- python3 -u tools/tune.py --log-n 20 --prec 64 --steps 5 --warmup 2 > gpurun_out/c1/pmc2.out 2>&1 || { tail gpurun_out/c1/pmc2.out; exit 1; }
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for d in ("gpurun_out/c1/pmc", "gpurun_out/c1/pmc2"):
    acc = defaultdict(lambda: defaultdict(float)); cnt = defaultdict(set)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_pass" in r["Kernel_Name"]:
                acc[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Kernel_Name"]].add(r.get("Dispatch_Id"))
    for k, c in acc.items():
        n = len(cnt[k])
        print(k[:60], n, {a: round(b / n) for a, b in sorted(c.items())})
PY
