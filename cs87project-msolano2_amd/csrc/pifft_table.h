// cs87project-msolano2_amd/csrc/pifft_table.h -- the registry of k_pass
// instantiations (one table per translation unit, see pifft_passes.hip).
#pragma once

namespace pifft {

struct PassKernel {
    int prec, R, C, mode, nts, lp;
    const void* fn;
    int nt;
    int lds_bytes;
    int vpt;  // values per thread (16; 32 for the packed fp32 passes)
};

}  // namespace pifft

#define PIFFT_NPART 8
