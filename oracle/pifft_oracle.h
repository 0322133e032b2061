/*
 * oracle/pifft_oracle.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the
 * reference pi-FFT (see pifft_oracle.c for the file:line map).  Used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the
 * product library.
 */
#ifndef PIFFT_ORACLE_H
#define PIFFT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float re, im; } oracle_cx_f32;   /* CPU.c:33-36 data_t */
typedef struct { double re, im; } oracle_cx_f64;  /* data_t with -Dfloat=double */

uint32_t oracle_ilog2_u64(uint64_t x);
uint64_t oracle_bit_reverse(uint64_t x, uint32_t m);
uint64_t oracle_splitmix64(uint64_t seed, uint64_t draw);
double oracle_u01(uint64_t seed, uint64_t draw);

oracle_cx_f32 oracle_omega_f32(uint64_t N, uint64_t k);
oracle_cx_f64 oracle_omega_f64(uint64_t N, uint64_t k);

int oracle_fft_f32(const oracle_cx_f32* in, oracle_cx_f32* out, uint64_t N, uint32_t P,
                   uint32_t nthreads, double* ms_tree, double* ms_cyl, double* ms_wall);
int oracle_fft_f64(const oracle_cx_f64* in, oracle_cx_f64* out, uint64_t N, uint32_t P,
                   uint32_t nthreads, double* ms_tree, double* ms_cyl, double* ms_wall);

int oracle_worker_f32(const oracle_cx_f32* in, oracle_cx_f32* out, uint64_t N, uint32_t P,
                      uint32_t q, double* ms_tree, double* ms_cyl);
int oracle_worker_f64(const oracle_cx_f64* in, oracle_cx_f64* out, uint64_t N, uint32_t P,
                      uint32_t q, double* ms_tree, double* ms_cyl);

int oracle_tree_segment_f32(const oracle_cx_f32* in, oracle_cx_f32* seg, uint64_t N,
                            uint32_t P, uint32_t q);
int oracle_tree_segment_f64(const oracle_cx_f64* in, oracle_cx_f64* seg, uint64_t N,
                            uint32_t P, uint32_t q);

void oracle_generate_f32(oracle_cx_f32* x, uint64_t count, uint64_t n, uint64_t seed,
                         uint64_t first);
void oracle_generate_f64(oracle_cx_f64* x, uint64_t count, uint64_t n, uint64_t seed,
                         uint64_t first);

int oracle_kat_f32(uint32_t P);

#ifdef __cplusplus
}
#endif

#endif
