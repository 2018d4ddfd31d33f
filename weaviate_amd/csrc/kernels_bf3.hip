// kernels_bf3.hip -- bf16 plane layout and LDS helpers shared by the block-key
// kernels (qs_kernels.hip).  (Round 1's three-term bf16 select kernels,
// k_mfma_select_bf3 / _bf3w, were superseded by the block-key path and
// removed; the tiled plane layout they introduced is the one the block-key
// pass streams.)
//
// Tiled bf16 plane: element (row, col) at
//   ((row / 256) * (dp / 16) + col / 16) * 4096 + (row % 256) * 16 + col % 16,
// so each 16-column slice of a 256-row tile is one contiguous 8 KiB run and a
// 32-row block of it one contiguous 1 KiB LDS-DMA piece.
#pragma once

namespace wv {
namespace {  // internal linkage: each runtime unit compiles the kernels it launches

typedef short bf16x8_t __attribute__((ext_vector_type(8)));

// element index of (row, col) in a tiled bf16 plane (dpad = the plane width dpb)
__host__ __device__ __forceinline__ int64_t bf3_plane_index(int64_t row, int col, int dpad) {
    return (((row >> 8) * (dpad >> 4) + (col >> 4)) << 12) + ((row & 255) << 4) + (col & 15);
}

__device__ __forceinline__ bf16x8_t lds_ld8bf(const unsigned char* p) {
    bf16x8_t v;
    const unsigned off = (unsigned)(size_t)((__attribute__((address_space(3))) const unsigned char*)p);
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(off));
    return v;
}

// Epilogue LDS traffic in inline asm: the LDS-DMA ring (global_load_lds)
// counts as pending LDS writes for the compiler, which then puts vmcnt(0) --
// a full drain of the ring -- before every LDS atomic/store and on every
// __syncthreads fence.  The candidate buffer, counters and flags are never a
// DMA target, so LDS ordering (lgkmcnt) is all these accesses need.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)((__attribute__((address_space(3))) const void*)p);
}
__device__ __forceinline__ int lds_add_rtn(int* p, int v) {
    int r;
    asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(lds_addr(p)), "v"(v) : "memory");
    return r;
}
__device__ __forceinline__ void lds_st(void* p, uint32_t v) {
    asm volatile("ds_write_b32 %0, %1" : : "v"(lds_addr(p)), "v"(v) : "memory");
}
// workgroup barrier ordering LDS only (no vmcnt drain of the DMA ring)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

// wave-uniform 8-byte read through the scalar cache (address 8-B aligned)
__device__ __forceinline__ uint64_t sload_u64(const void* p) {
    // p is wave-uniform but derived from threadIdx: move it to SGPRs
    const uint64_t pi = (uint64_t)p;
    const uint64_t up = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(pi >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)pi);
    uint64_t v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(up) : "memory");
    return v;
}

// ds_read_b128 at LDS byte address base + OFF (immediate offset field)
template <int OFF>
__device__ __forceinline__ bf16x8_t lds_ld8bf_o(unsigned base) {
    bf16x8_t v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(OFF));
    return v;
}

}  // namespace
}  // namespace wv
