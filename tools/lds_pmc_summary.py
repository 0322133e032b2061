#!/usr/bin/env python3
"""tools/lds_pmc_summary.py <rocprofv3 -d dir> -- per-kernel LDS bank-conflict
ratio (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE) and scratch bytes from a
`rocprofv3 --pmc` counter collection (summed over the kernel's dispatches)."""
import csv
import glob
import sys
from collections import defaultdict

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
acc = defaultdict(lambda: defaultdict(float))
scratch = {}
for r in rows:
    k = r.get("Kernel_Name", "?")
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    scratch[k] = r.get("Scratch_Size", r.get("Private_Segment_Size", "?"))
for k, c in sorted(acc.items()):
    if "k_pass" not in k and "k_tree" not in k:
        continue
    act = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
    ratio = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / act if act else 0.0
    print(f"{ratio:.3f}  conflict/active  unaligned {c.get('SQ_LDS_UNALIGNED_STALL', 0):.0f}  scratch {scratch[k]}  {k}")
