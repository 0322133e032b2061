"""oracle/integrate_ref.py -- TEST INFRASTRUCTURE ONLY (this container only).

Demonstrates INTEGRATION.md section 2 on the reference itself: copies the
reference CPU source to a temporary directory (never into the repository),
replaces the pthread fan-out of its run() (CPU.c:335-360) with the libpifft
calls shown in INTEGRATION.md, and compiles it into
oracle/_ref/fourier-parallel-pi-cpu-pthreads-gpu{,-f64}, linked against the
in-tree libpifft.so.  tests/test_gpu_parity.py runs that binary (the
reference's own main/setup_from_args/initialize_data/verify_results with the
MI355X backend).
"""
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = "/root/reference/benchmark/fourier/parallel/pi/cpu/pthreads/fourier-parallel-pi-cpu-pthreads.c"

PATCH = r'''  {
  pifft_plan* plan;
  double ms1, ms2;
  int prec = sizeof(data_t) == 16 ? PIFFT_F64 : PIFFT_F32;   /* -Dfloat=double -> fp64 */
  if (pifft_plan_create(&plan, t->N, t->P, 1, prec)) {       /* CPU.c:139-198 rules */
    stderr_out("%s\n", pifft_last_error());
    cleanup_data(t);
    goto err;
  }
  if (pifft_execute(plan, t->in, t->out, &ms1, &ms2)) {      /* all P workers, natural-order out */
    stderr_out("%s\n", pifft_last_error());
    pifft_plan_destroy(plan);
    cleanup_data(t);
    goto err;
  }
  pifft_plan_destroy(plan);
  if (!t->test_mode) {                                         /* CPU.c:485-492 */
    if (!t->no_header) print_out("n\tp\ttime (total)\ttime (stage 1)\ttime (stage 2)\n");
    print_out("%u\t%u\t%lf\t%lf\t%lf\n", t->N, t->P, ms1 + ms2, ms1, ms2);
  }
  }

'''


def main() -> int:
    if not os.path.exists(REF):
        print("reference source not present; nothing to build")
        return 0
    lib = os.path.join(ROOT, "cs87project-msolano2_amd")
    out_dir = os.path.join(HERE, "_ref")
    os.makedirs(out_dir, exist_ok=True)
    src = open(REF).read()
    a = src.index("  // Spawn P pthreads, each running 'run_thread'")
    b = src.index("  // If in test mode, print out the result, and verify that it is correct.")
    src = src[:a] + PATCH + src[b:]
    src = src.replace("#include <pthread.h>", '#include <pthread.h>\n#include "pifft.h"', 1)
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "ref_gpu.c")
        with open(path, "w") as f:
            f.write(src)
        for suffix, extra in (("", []), ("-f64", ["-Dfloat=double"])):
            exe = os.path.join(out_dir, "fourier-parallel-pi-cpu-pthreads-gpu" + suffix)
            subprocess.run(["gcc", "-O2", "-w", "-fopenmp", "-pthread", *extra, path, "-I", os.path.join(ROOT, "include"),
                            "-L", lib, "-lpifft", "-Wl,-rpath," + lib, "-lm", "-o", exe], check=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
