// tests/native/gather_schedule_main.cpp -- prints pifft_allgather's copy
// schedule (csrc/pifft_gather.h) for a mocked device list, as JSON, for
// tests/test_gather_schedule.py (host-only: no HIP, no GPU).
//   usage: gather_schedule N P batch dst_mask dev0:q0:nq dev1:q0:nq ...
#include <stdio.h>
#include <stdlib.h>

#include "../../cs87project-msolano2_amd/csrc/pifft_gather.h"

int main(int argc, char** argv) {
    if (argc < 6) return 2;
    const uint64_t N = strtoull(argv[1], nullptr, 10);
    const uint64_t P = strtoull(argv[2], nullptr, 10);
    const uint32_t batch = (uint32_t)strtoul(argv[3], nullptr, 10);
    const uint64_t mask = strtoull(argv[4], nullptr, 0);
    std::vector<pifft::GatherSrc> srcs;
    std::vector<bool> has;
    for (int a = 5; a < argc; a++) {
        int dev = 0;
        unsigned q0 = 0, nq = 0;
        if (sscanf(argv[a], "%d:%u:%u", &dev, &q0, &nq) != 3) return 2;
        srcs.push_back({dev, q0, nq});
        has.push_back((mask >> (a - 5)) & 1);
    }
    const pifft::GatherSchedule g = pifft::gather_schedule(srcs, has, N, N / P, batch);
    printf("{\"streams\": %d, \"peer\": [", g.streams);
    for (size_t i = 0; i < g.peer.size(); i++) printf("%s[%d, %d]", i ? ", " : "", g.peer[i].first, g.peer[i].second);
    printf("], \"copies\": [");
    for (size_t i = 0; i < g.copies.size(); i++) {
        const auto& c = g.copies[i];
        printf("%s{\"dst\": %d, \"src\": %d, \"stream\": %d, \"dst_off\": %llu, \"src_off\": %llu, \"elems\": %llu, "
               "\"peer\": %s}", i ? ", " : "", c.dst, c.src, c.stream, (unsigned long long)c.dst_off,
               (unsigned long long)c.src_off, (unsigned long long)c.elems, c.peer ? "true" : "false");
    }
    printf("]}\n");
    return 0;
}
