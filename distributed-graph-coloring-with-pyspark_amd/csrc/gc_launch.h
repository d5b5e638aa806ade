// gc_launch.h -- host-side view of the device state and the kernel launch wrappers.
#pragma once
#include <hip/hip_runtime.h>
#include "gc_internal.h"

struct GcDevView {
    int n;
    long long nnz;
    const long long* rp;
    const int* col;
    const int* deg;
    const long long* trp;
    const int* tcol;
    int* color;
    int* cround;
    ull* key;
    unsigned char* jp;
    unsigned int* inF;
    DevCtl* ctl;
};

void gcl_init(const GcDevView& d, int* seed_light, int grid, hipStream_t s);
void gcl_seed_prep(const GcDevView& d, int* sl, int* sh, hipStream_t s);
void gcl_propose_light(const GcDevView& d, const int* list, const ull* cnt, int* heavy, int* wide, long long k,
                       int grid, hipStream_t s);
void gcl_propose_block(const GcDevView& d, const int* la, const ull* ca, const int* lb, const ull* cb, long long k,
                       int words, int grid, hipStream_t s);
void gcl_resolve_light(const GcDevView& d, const int* list, const ull* cnt, int skip_heavy, int* und, ull* und_cnt,
                       int kclass, int grid, hipStream_t s);
void gcl_resolve_block(const GcDevView& d, const int* list, const ull* cnt, int* und, ull* und_cnt, int grid,
                       hipStream_t s);
void gcl_commit_light(const GcDevView& d, const int* list, const ull* cnt, int skip_heavy, int* next, ull* next_cnt,
                      int round, int grid, hipStream_t s);
void gcl_commit_block(const GcDevView& d, const int* list, const ull* cnt, int* next, ull* next_cnt, int round,
                      int grid, hipStream_t s);
void gcl_unc_compact(const GcDevView& d, int* list, ull* cnt, int* parent, ull* best, int grid, hipStream_t s);
void gcl_cc_hook(const GcDevView& d, const int* list, const ull* cnt, int* parent, int grid, hipStream_t s);
void gcl_cc_best(const GcDevView& d, const int* list, const ull* cnt, int* parent, ull* best, int grid,
                 hipStream_t s);
void gcl_cc_seeds(const GcDevView& d, const int* list, const ull* cnt, int* parent, const ull* best, int* sl,
                  int* sh, int grid, hipStream_t s);
void gcl_validate(const GcDevView& d, const int* colors, int grid, hipStream_t s);
void gcl_degrees(const long long* rp, int n, int* deg, ull* maxdeg, int grid, hipStream_t s);
