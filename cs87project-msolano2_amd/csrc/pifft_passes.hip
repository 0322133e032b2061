// cs87project-msolano2_amd/csrc/pifft_passes.hip -- one slice of the k_pass
// instantiations (compiled PIFFT_NPART times with -DPIFFT_PART=k, in parallel).
#include "pifft_kernels.h"
#include "pifft_table.h"

#if !defined(PIFFT_PART) || !defined(PIFFT_INC)
#error "compile with -DPIFFT_PART=<k> -DPIFFT_INC='\"pifft_instances_<k>.inc\"'"
#endif
#define PIFFT_CAT2(a, b) a##b
#define PIFFT_CAT(a, b) PIFFT_CAT2(a, b)

using namespace pifft;

#define PKV(T, PREC, R, C, MODE, NTS, LP, VPT)                                                          \
    PassKernel {                                                                                        \
        PREC, R, C, MODE, NTS, LP, reinterpret_cast<const void*>(&k_pass<T, R, C, MODE, NTS, LP, VPT>), \
            PassCfg<R, C, VPT>::NT, pass_lds_bytes<T, R, C, MODE, VPT>(), VPT                           \
    }
#define PK(T, PREC, R, C, MODE, NTS, LP) PKV(T, PREC, R, C, MODE, NTS, LP, 16)

namespace {
const PassKernel kTable[] = {
#include PIFFT_INC
};
}  // namespace

extern "C" const PassKernel* PIFFT_CAT(pifft_pass_table_, PIFFT_PART)(int* n) {
    *n = (int)(sizeof(kTable) / sizeof(kTable[0]));
    return kTable;
}
