// fetode_xrank.h — the cross-rank exchange records of the trajectory-sharded device-resident
// dopri5 solvers (fetode_integrate_dopri5_xrank, fetode_wide_dopri5_xrank): every rank's kernel
// writes its norm records into every peer's inbox (fine-grained device memory, IPC-mapped into each
// rank: remote stores over xGMI) and polls its own inbox for the peers' round tags.  Device code
// only; included inside each file's anonymous namespace.
#pragma once

// System-scope (sc0 sc1: write-through to memory / read past every cache) records for the
// cross-rank exchange: the payload lands before the tag that publishes it (vmcnt(0) between).
typedef unsigned xr_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void xr_st16(double* p, double v0, double v1) {
  const unsigned long long a = __double_as_longlong(v0), b = __double_as_longlong(v1);
  const xr_u32x4 v = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void xr_st_tag(double* p, unsigned long long tag) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 v = {(unsigned)tag, (unsigned)(tag >> 32)};
  asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ unsigned long long xr_ld_tag(const double* p) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  u32x2 v;
  asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return ((unsigned long long)v.y << 32) | v.x;
}
__device__ __forceinline__ void xr_ld16(const double* p, double& v0, double& v1) {
  xr_u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  v0 = __longlong_as_double(((unsigned long long)v.y << 32) | v.x);
  v1 = __longlong_as_double(((unsigned long long)v.w << 32) | v.z);
}

// inbox: (2 parity, 64 items) {v0, v1} records, then (2 parity, 64 ranks) tags (fetode_xrank_inbox_bytes)
__device__ __forceinline__ double* xr_rec(double* inbox, unsigned par, int item) { return inbox + 2 * (64 * par + item); }
__device__ __forceinline__ double* xr_tagp(double* inbox, unsigned par, int rank) {
  return inbox + 2 * 2 * 64 + (64 * par + rank);
}
