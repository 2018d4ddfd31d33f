// multi.hip -- the sharded exact search behind the C ABI (wv_multi_*).
//
// Weaviate searches every shard a node holds inside one Go process and merges
// the shard results there (adapters/repos/db/index.go:1928-2071).  Here one
// process drives every shard it holds -- one per GPU, or several on one GPU
// for tests -- through the two-phase protocol of DESIGN.md §4, with the
// collectives issued by the library itself on a transport it owns:
//   * RCCL (dlopen'ed at run time, the copy already in the process when there
//     is one): one communicator per local shard; several processes (one per
//     GPU, the bench under torch.distributed.run) share a world through a
//     128-byte unique id the host passes around, one process may hold every
//     GPU of the node (ncclCommInitRank for each in one group);
//   * in-process device copies: every rank of the world is a shard of this
//     process (devices may repeat), for one-GPU tests and the 8-rank cost
//     model (option "sim": ranks run stage by stage, each timed alone).
// Every shard holds a contiguous doc-id range [r * id_stride, (r+1) * id_stride)
// (the last rank: to the end), so the id-ordered scan of one reference index
// is the concatenation of the rank scans in rank order, and the result equals
// the single index's bit for bit (ids, distances, tie order).
//
// One search (stage-major over the local shards, all device work async):
//   1. phase 1 (wv_index_shard_phase1): block keys + candidate selection;
//      a shard off the block-key path contributes +inf keys, eps 0;
//   2. all-gather of the k+1 smallest keys and eps; phase 2 (global cut +
//      exact rows) or the one-shot local search (mode 1) off the path;
//   3. all-gather of the lists; wv_merge_shards; ascending flagged list
//      (one host sync for its length);
//   4. flagged queries, k < 64: the parallel replay -- rank 0 from empty
//      heaps, rank r >= 1 from k copies of T_r (k_prefix_bound) recording its
//      insertions; all-gather of the records; wv_heap_merge_records (one host
//      sync for the overflow count; overflowed queries take the serial chain);
//      k >= 64: the serial chain over the flags, one broadcast per hop.
#include "rt_index.h"

#include <dlfcn.h>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <thread>
#include <memory>
#include <rccl/rccl.h>  // types only: the library is bound at run time

namespace {

// ---------------------------------------------------------------------------
// RCCL, bound at run time
// ---------------------------------------------------------------------------
struct RcclApi {
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclAllGather) AllGather = nullptr;
    decltype(&ncclBroadcast) Broadcast = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    std::string err;
    bool ok = false;
};

const RcclApi& rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        const char* env = getenv("WV_RCCL_LIB");
        if (env && *env) h = dlopen(env, RTLD_NOW | RTLD_LOCAL);
        // a copy already mapped into the process (torch's) is reused: one RCCL per process
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            api.err = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return;
        }
#define WV_SYM(n)                                                      \
    api.n = (decltype(api.n))dlsym(h, "nccl" #n);                      \
    if (!api.n) { api.err = "librccl.so.1 lacks nccl" #n; return; }
        WV_SYM(GetUniqueId) WV_SYM(CommInitRank) WV_SYM(CommDestroy) WV_SYM(AllGather) WV_SYM(Broadcast)
        WV_SYM(GroupStart) WV_SYM(GroupEnd) WV_SYM(GetErrorString)
#undef WV_SYM
        api.ok = true;
    });
    return api;
}

#define RCCLCHK(x)                                                                                   \
    do {                                                                                             \
        ncclResult_t r_ = (x);                                                                       \
        if (r_ != ncclSuccess) return set_err(WV_ERR_HIP, "%s: %s", #x, rccl().GetErrorString(r_)); \
    } while (0)

// ---------------------------------------------------------------------------
// transports: collectives over the world, issued for every local shard at
// once on the shards' streams (send/recv/buf: field-major, [f * nlocal + i])
// ---------------------------------------------------------------------------
struct Transport {
    std::vector<int> dev;
    std::vector<hipStream_t> s;
    virtual ~Transport() {}
    // local shard i sends bytes[f] from send[f][i]; recv[f][i] gets [world][bytes[f]]
    virtual int all_gather(int nf, const void* const* send, void* const* recv, const size_t* bytes) = 0;
    // buf[f][root] -> buf[f][i] of every rank
    virtual int broadcast(int nf, void* const* buf, const size_t* bytes, int root) = 0;
};

// every rank of the world is a local shard: device-to-device copies, ordered by
// events (each receiver waits for every sender's stream; every sender then
// waits for the receivers' copies before it may overwrite its buffer)
struct LocalTransport : Transport {
    std::vector<hipEvent_t> ready, done;
    ~LocalTransport() override {
        for (size_t i = 0; i < dev.size(); i++) {
            hipSetDevice(dev[i]);
            if (ready[i]) hipEventDestroy(ready[i]);
            if (done[i]) hipEventDestroy(done[i]);
        }
    }
    int init() {
        ready.assign(dev.size(), nullptr);
        done.assign(dev.size(), nullptr);
        for (size_t i = 0; i < dev.size(); i++) {
            HIPCHK(hipSetDevice(dev[i]));
            HIPCHK(hipEventCreateWithFlags(&ready[i], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
            for (size_t j = 0; j < dev.size(); j++)
                if (dev[j] != dev[i]) {
                    hipError_t e = hipDeviceEnablePeerAccess(dev[j], 0);
                    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return set_err(WV_ERR_HIP, "peer access %d -> %d: %s", dev[i], dev[j], hipGetErrorString(e));
                    (void)hipGetLastError();
                }
        }
        return WV_OK;
    }
    int copy(void* dst, int ddev, const void* src, int sdev, size_t b, hipStream_t st) {
        if (b == 0 || dst == src) return WV_OK;
        if (ddev == sdev) HIPCHK(hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToDevice, st));
        else HIPCHK(hipMemcpyPeerAsync(dst, ddev, src, sdev, b, st));
        return WV_OK;
    }
    int all_gather(int nf, const void* const* send, void* const* recv, const size_t* bytes) override {
        const int n = (int)dev.size();
        for (int i = 0; i < n; i++) {
            HIPCHK(hipSetDevice(dev[i]));
            HIPCHK(hipEventRecord(ready[i], s[i]));
        }
        for (int j = 0; j < n; j++) {
            HIPCHK(hipSetDevice(dev[j]));
            for (int i = 0; i < n; i++)
                if (i != j) HIPCHK(hipStreamWaitEvent(s[j], ready[i], 0));
            for (int f = 0; f < nf; f++)
                for (int i = 0; i < n; i++) {
                    int rc = copy((char*)recv[f * n + j] + (size_t)i * bytes[f], dev[j], send[f * n + i], dev[i],
                                  bytes[f], s[j]);
                    if (rc) return rc;
                }
            HIPCHK(hipEventRecord(done[j], s[j]));
        }
        for (int i = 0; i < n; i++) {
            HIPCHK(hipSetDevice(dev[i]));
            for (int j = 0; j < n; j++)
                if (i != j) HIPCHK(hipStreamWaitEvent(s[i], done[j], 0));
        }
        return WV_OK;
    }
    int broadcast(int nf, void* const* buf, const size_t* bytes, int root) override {
        const int n = (int)dev.size();
        HIPCHK(hipSetDevice(dev[root]));
        HIPCHK(hipEventRecord(ready[root], s[root]));
        for (int j = 0; j < n; j++) {
            if (j == root) continue;
            HIPCHK(hipSetDevice(dev[j]));
            HIPCHK(hipStreamWaitEvent(s[j], ready[root], 0));
            for (int f = 0; f < nf; f++) {
                int rc = copy(buf[f * n + j], dev[j], buf[f * n + root], dev[root], bytes[f], s[j]);
                if (rc) return rc;
            }
            HIPCHK(hipEventRecord(done[j], s[j]));
        }
        HIPCHK(hipSetDevice(dev[root]));
        for (int j = 0; j < n; j++)
            if (j != root) HIPCHK(hipStreamWaitEvent(s[root], done[j], 0));
        return WV_OK;
    }
};

// RCCL: one communicator per local shard, every call of one collective in one
// group (a single host thread drives several devices)
struct RcclTransport : Transport {
    std::vector<ncclComm_t> comm;
    ~RcclTransport() override {
        for (size_t i = 0; i < comm.size(); i++)
            if (comm[i]) { hipSetDevice(dev[i]); rccl().CommDestroy(comm[i]); }
    }
    int init(int world, int rank0, const void* uid) {
        const RcclApi& a = rccl();
        if (!a.ok) return set_err(WV_ERR_UNSUPPORTED, "%s", a.err.c_str());
        ncclUniqueId id;
        if (uid) memcpy(&id, uid, sizeof(id));
        else RCCLCHK(a.GetUniqueId(&id));  // the whole world is local
        comm.assign(dev.size(), nullptr);
        RCCLCHK(a.GroupStart());
        for (size_t i = 0; i < dev.size(); i++) {
            HIPCHK(hipSetDevice(dev[i]));
            ncclResult_t r = a.CommInitRank(&comm[i], world, id, rank0 + (int)i);
            if (r != ncclSuccess) { a.GroupEnd(); return set_err(WV_ERR_HIP, "ncclCommInitRank: %s", a.GetErrorString(r)); }
        }
        RCCLCHK(a.GroupEnd());
        return WV_OK;
    }
    int all_gather(int nf, const void* const* send, void* const* recv, const size_t* bytes) override {
        const RcclApi& a = rccl();
        const int n = (int)dev.size();
        RCCLCHK(a.GroupStart());
        for (int f = 0; f < nf; f++)
            for (int i = 0; i < n; i++) {
                ncclResult_t r = a.AllGather(send[f * n + i], recv[f * n + i], bytes[f], ncclChar, comm[i], s[i]);
                if (r != ncclSuccess) { a.GroupEnd(); return set_err(WV_ERR_HIP, "ncclAllGather: %s", a.GetErrorString(r)); }
            }
        RCCLCHK(a.GroupEnd());
        return WV_OK;
    }
    int broadcast(int nf, void* const* buf, const size_t* bytes, int root) override {
        const RcclApi& a = rccl();
        const int n = (int)dev.size();
        RCCLCHK(a.GroupStart());
        for (int f = 0; f < nf; f++)
            for (int i = 0; i < n; i++) {
                ncclResult_t r = a.Broadcast(buf[f * n + i], buf[f * n + i], bytes[f], ncclChar, root, comm[i], s[i]);
                if (r != ncclSuccess) { a.GroupEnd(); return set_err(WV_ERR_HIP, "ncclBroadcast: %s", a.GetErrorString(r)); }
            }
        RCCLCHK(a.GroupEnd());
        return WV_OK;
    }
};

// one local shard; collectives staged through host memory to the caller's
// functions (synchronous: the shard's stream is drained first)
struct HostTransport : Transport {
    int world = 1, rank = 0;
    wv_host_allgather_fn ag = nullptr;
    wv_host_broadcast_fn bc = nullptr;
    void* user = nullptr;
    std::vector<unsigned char> hs, hr;
    int all_gather(int nf, const void* const* send, void* const* recv, const size_t* bytes) override {
        HIPCHK(hipSetDevice(dev[0]));
        for (int f = 0; f < nf; f++) {
            hs.resize(std::max<size_t>(bytes[f], 1));
            hr.resize(std::max<size_t>(bytes[f] * world, 1));
            HIPCHK(hipMemcpyAsync(hs.data(), send[f], bytes[f], hipMemcpyDeviceToHost, s[0]));
            HIPCHK(hipStreamSynchronize(s[0]));
            if (ag(hs.data(), hr.data(), (int64_t)bytes[f], user) != 0)
                return set_err(WV_ERR_HIP, "host transport: all-gather callback failed");
            HIPCHK(hipMemcpyAsync(recv[f], hr.data(), bytes[f] * world, hipMemcpyHostToDevice, s[0]));
            HIPCHK(hipStreamSynchronize(s[0]));
        }
        return WV_OK;
    }
    int broadcast(int nf, void* const* buf, const size_t* bytes, int root) override {
        HIPCHK(hipSetDevice(dev[0]));
        for (int f = 0; f < nf; f++) {
            hs.resize(std::max<size_t>(bytes[f], 1));
            if (rank == root) {
                HIPCHK(hipMemcpyAsync(hs.data(), buf[f], bytes[f], hipMemcpyDeviceToHost, s[0]));
                HIPCHK(hipStreamSynchronize(s[0]));
            }
            if (bc(hs.data(), (int64_t)bytes[f], root, user) != 0)
                return set_err(WV_ERR_HIP, "host transport: broadcast callback failed");
            if (rank != root) {
                HIPCHK(hipMemcpyAsync(buf[f], hs.data(), bytes[f], hipMemcpyHostToDevice, s[0]));
                HIPCHK(hipStreamSynchronize(s[0]));
            }
        }
        return WV_OK;
    }
};

// ---------------------------------------------------------------------------
// small kernels of the protocol
// ---------------------------------------------------------------------------
__global__ void k_mfill_f32(float* __restrict__ p, int64_t n, float v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// flags[n] != 0 -> their indices, ascending (one workgroup: the list and its
// order are identical on every rank, which the record all-gather relies on);
// src != null maps position i to src[i]
__global__ __launch_bounds__(1024) void k_list_ascending(const int32_t* __restrict__ flags, const int32_t* __restrict__ src,
                                                         int n, int32_t* __restrict__ list, int32_t* __restrict__ count) {
    __shared__ int wsum[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int base = 0;
    for (int c0 = 0; c0 < n; c0 += 1024) {
        const int i = c0 + t;
        const bool f = i < n && flags[i] != 0;
        const uint64_t m = __ballot(f);
        if (lane == 0) wsum[w] = __popcll(m);
        __syncthreads();
        int before = 0, tot = 0;
        for (int j = 0; j < 16; j++) {
            const int v = wsum[j];
            before += j < w ? v : 0;
            tot += v;
        }
        if (f) list[base + before + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0))] =
            src ? src[i] : i;
        base += tot;
        __syncthreads();
    }
    if (t == 0) *count = base;
}

// k-th smallest (1-based) of v[0..n) held in LDS by one workgroup; +inf when n < k
__device__ float kth_smallest(const float* v, int n, int k, float* slot) {
    if (threadIdx.x == 0) *slot = __builtin_inff();
    __syncthreads();
    if (n >= k)
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const float x = v[i];
            int lt = 0, le = 0;
            for (int j = 0; j < n; j++) {
                lt += v[j] < x;
                le += v[j] <= x;
            }
            if (lt < k && k <= le) *slot = x;  // every writer holds the same value
        }
    __syncthreads();
    const float r = *slot;
    __syncthreads();
    return r;
}

// the fake heap of listed query ql[li] on rank r >= 1 (sharded.py prefix_bound +
// fake_heaps): T_r = min(k-th smallest exact distance of the unflagged lists of
// ranks < r, k-th smallest block bound A + eps of their phase-1 keys) -- each
// an upper bound of the real heap top at rank r's first row; the heap is k
// copies of T_r (ids -1), empty when T_r is infinite
// (the compressed R-heaps: ql, gc, gf NULL -- every query, every one of the k1
// gathered block minima a bound of one distinct row)
__global__ __launch_bounds__(256) void k_prefix_bound(int r, const int32_t* __restrict__ ql, int F, int k, int k1, int64_t nq,
                                                      const float* __restrict__ gd, const int32_t* __restrict__ gc,
                                                      const int32_t* __restrict__ gf, const float* __restrict__ gA,
                                                      const float* __restrict__ gE, uint64_t* __restrict__ oi,
                                                      float* __restrict__ od, int32_t* __restrict__ on) {
    extern __shared__ float pbv[];
    __shared__ float slot;
    const int li = blockIdx.x;
    if (li >= F) return;
    const int64_t q = ql ? ql[li] : li;
    const int n = r * k1;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int rr = i / k1, j = i - rr * k1;
        const int64_t row = (int64_t)rr * nq + q;
        const bool ok = (!gc || j < gc[row]) && (!gf || gf[row] == 0);
        pbv[i] = ok ? gd[row * k1 + j] : __builtin_inff();
    }
    __syncthreads();
    float T = kth_smallest(pbv, n, k, &slot);
    if (gA) {
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const int rr = i / k1, j = i - rr * k1;
            const int64_t row = (int64_t)rr * nq + q;
            pbv[i] = gA[row * k1 + j] + gE[row];
        }
        __syncthreads();
        T = fminf(T, kth_smallest(pbv, n, k, &slot));
    }
    for (int j = threadIdx.x; j < k; j += blockDim.x) {
        oi[(int64_t)li * k + j] = ~0ull;
        od[(int64_t)li * k + j] = T;
    }
    if (threadIdx.x == 0) on[li] = isinf(T) ? 0 : k;
}

// heap state [F][k] -> the first k entries of record rows [F][cap]
__global__ void k_state_to_rec(const uint64_t* __restrict__ ti, const float* __restrict__ td, const int32_t* __restrict__ tn,
                               int F, int k, int cap, uint64_t* __restrict__ ri, float* __restrict__ rd,
                               int32_t* __restrict__ rn) {
    const int li = blockIdx.x;
    for (int j = threadIdx.x; j < k; j += blockDim.x) {
        ri[(int64_t)li * cap + j] = ti[(int64_t)li * k + j];
        rd[(int64_t)li * cap + j] = td[(int64_t)li * k + j];
    }
    if (threadIdx.x == 0) rn[li] = tn[li];
}

// listed results [F][k] -> rows ql[li] of the merged results [nq][k]
__global__ void k_scatter_rows(const int32_t* __restrict__ ql, int F, int k, const uint64_t* __restrict__ fi,
                               const float* __restrict__ fd, const int32_t* __restrict__ fn, uint64_t* __restrict__ oi,
                               float* __restrict__ od, int32_t* __restrict__ on) {
    const int li = blockIdx.x;
    const int64_t q = ql[li];
    for (int j = threadIdx.x; j < k; j += blockDim.x) {
        oi[q * k + j] = fi[(int64_t)li * k + j];
        od[q * k + j] = fd[(int64_t)li * k + j];
    }
    if (threadIdx.x == 0) on[q] = fn[li];
}

// order-preserving float <-> u32 keys (NaN above +inf, as torch.topk ranks it)
__device__ inline uint32_t ord_key(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float ord_val(uint32_t k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k); }

// per query the R smallest of its nblk block minima (sharded.py quant_bounds'
// topk, unordered: only their R-th smallest is used), +inf padded.  One
// workgroup per query: a 4-pass 8-bit radix select of the R-th smallest key,
// then every value below it and as many copies of it as complete R.
__global__ __launch_bounds__(256) void k_smallest_r(const float* __restrict__ bm, int64_t nblk, int R,
                                                    float* __restrict__ out) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t s_prefix, s_need, s_cnt;
    const int q = blockIdx.x;
    const float* B = bm + (int64_t)q * nblk;
    float* O = out + (int64_t)q * R;
    if (nblk <= R) {
        for (int i = threadIdx.x; i < R; i += blockDim.x) O[i] = i < nblk ? B[i] : __builtin_inff();
        return;
    }
    if (threadIdx.x == 0) { s_prefix = 0; s_need = (uint32_t)R; s_cnt = 0; }
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
        __syncthreads();
        const uint32_t prefix = s_prefix;
        const uint32_t hi_mask = shift == 24 ? 0u : (0xffffffffu << (shift + 8));
        for (int64_t b = threadIdx.x; b < nblk; b += blockDim.x) {
            const uint32_t key = ord_key(B[b]);
            if ((key & hi_mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t c = 0, need = s_need;
            for (int dgt = 0; dgt < 256; dgt++) {
                if (c + hist[dgt] >= need) { s_prefix = prefix | ((uint32_t)dgt << shift); s_need = need - c; break; }
                c += hist[dgt];
            }
        }
        __syncthreads();
    }
    const uint32_t T = s_prefix;  // the R-th smallest key; s_need of its copies complete the R
    const int below = R - (int)s_need;
    for (int64_t b = threadIdx.x; b < nblk; b += blockDim.x) {
        const float v = B[b];
        if (ord_key(v) < T) O[atomicAdd(&s_cnt, 1u)] = v;
    }
    for (int i = below + threadIdx.x; i < R; i += blockDim.x) O[i] = ord_val(T);
}

// the merged R-heap extracted ascending -> its pop order (max first, flat/index.go:509-523)
__global__ void k_rev_rows(const uint64_t* __restrict__ asc, const int32_t* __restrict__ n, int R,
                           uint64_t* __restrict__ out) {
    const int li = blockIdx.x;
    const int m = n[li];
    for (int j = threadIdx.x; j < R; j += blockDim.x)
        out[(int64_t)li * R + j] = j < m ? asc[(int64_t)li * R + (m - 1 - j)] : ~0ull;
}

__global__ void k_iota32(int32_t* __restrict__ p, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = (int32_t)i;
}

}  // namespace

// ---------------------------------------------------------------------------
// host threads: one per local shard beyond the first, so the stages of the
// shards of one process are issued in parallel (a shard's stage is a few
// dozen launches, ~0.4 ms of host time: issued one shard after another, the
// last of 8 GPUs would start its stage ~3 ms after the first)
// ---------------------------------------------------------------------------
struct StagePool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv, done;
    std::function<void(int)> task;
    uint64_t gen = 0;
    int pending = 0;
    bool stop = false;
    explicit StagePool(int n) {
        for (int i = 1; i < n; i++)
            th.emplace_back([this, i] {
                uint64_t seen = 0;
                for (;;) {
                    std::function<void(int)> t;
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [&] { return stop || gen != seen; });
                        if (stop) return;
                        seen = gen;
                        t = task;
                    }
                    t(i);
                    std::lock_guard<std::mutex> lk(mu);
                    if (--pending == 0) done.notify_one();
                }
            });
    }
    ~StagePool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
    }
    // fn(i) for every shard: 1.. on the pool's threads, 0 on the caller's
    void run(int n, const std::function<void(int)>& fn) {
        {
            std::lock_guard<std::mutex> lk(mu);
            task = fn;
            pending = n - 1;
            gen++;
        }
        cv.notify_all();
        fn(0);
        std::unique_lock<std::mutex> lk(mu);
        done.wait(lk, [&] { return pending == 0; });
    }
};

// ---------------------------------------------------------------------------
// the multi-shard index
// ---------------------------------------------------------------------------
enum { ST_PHASE1, ST_PHASE2, ST_MERGE, ST_REPLAY, ST_MERGE_REC, ST_CHAIN, ST_XFER, ST_N };

struct MRank {
    wv_index* idx = nullptr;
    int dev = 0, rank = 0;
    hipStream_t s = nullptr;
    hipEvent_t e_out = nullptr, e_in = nullptr;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    const float* qp = nullptr;
    bool off = false;
    DBuf q, topA, eps, gA, gE, ids, dd, cnt, flg, gi, gd, gc, gf, oi, od, on, of, ql, nl, fki, fkd, fkn, ti, td, tn, ri, rd,
        rn, gri, grd, grn, sti, std_, fi, fd, fn, un, ul, nu, ci[2], cd[2], cn[2];
    // compressed searches (BQ, PQ / SQ / RQ): bounds, candidates, rescoring
    DBuf bm, bnd, gbnd, cand, E, gEall, iota, mb, gmb;
    int64_t nblk = 0;
    // a filtered search: the shard's own present bitmap while the allow bitmap stands in
    uint32_t* saved_present = nullptr;
    int64_t saved_npresent = 0;
};

struct wv_multi {
    std::mutex mu;
    int world = 1, rank0 = 0, nl = 1, kind = WV_TRANSPORT_LOCAL;
    uint64_t id_stride = 0;
    std::vector<std::unique_ptr<MRank>> r;
    std::unique_ptr<Transport> tr;
    std::unique_ptr<StagePool> pool;  // option host_threads (default 1 with several local shards)
    hipEvent_t e_call = nullptr;
    int32_t* pin = nullptr;  // pinned host words: flagged count, overflow count
    int sim = 0;
    int sim_rev = 0;  // option sim_rev: option sim times the shards in reverse order (is a slow first shard the shard or its slot?)
    // host time of the last search: spent issuing work vs blocked in the host syncs (us)
    double host_total_us = 0, host_wait_us = 0;
    int rec_cap = 0;  // option rec_cap (tests): replay record capacity, 0 = max(256, 16 k) (exact), 2R (BQ), 2R + 64 (quantized)
    int force_chain = 0;  // option chain (tests): compressed searches take the serial chain
    double stage_ms[ST_N][64] = {};  // option sim: stage times summed over sim_n searches
    int64_t sim_n = 0;
    int64_t n_search = 0, n_flagged = 0, n_overflow = 0, n_chain = 0, last_flagged = 0, last_overflow = 0;
};

namespace {

int owner_rank(const wv_multi* m, uint64_t id) {
    const uint64_t r = m->id_stride ? id / m->id_stride : 0;
    return (int)std::min<uint64_t>(r, (uint64_t)(m->world - 1));
}

// a host sync of the protocol, its blocked time accounted (wv_multi_stats)
hipError_t host_sync(wv_multi* m, hipStream_t s) {
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = hipStreamSynchronize(s);
    m->host_wait_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    return e;
}

// issue one stage on every local shard; with option sim every shard's part is
// timed alone (HIP events, then a sync before the next shard)
template <class Fn>
int run_stage(wv_multi* m, int st, Fn fn) {
    if (m->pool && !m->sim) {
        // every shard's part on its own host thread; a failure's text moves to
        // the caller's thread (wv_last_error is per thread)
        std::vector<int> rc((size_t)m->nl, WV_OK);
        std::vector<std::string> err((size_t)m->nl);
        m->pool->run(m->nl, [&](int i) {
            MRank& R = *m->r[i];
            hipError_t e = hipSetDevice(R.dev);
            rc[(size_t)i] = e == hipSuccess ? fn(R, i) : set_err(WV_ERR_HIP, "hipSetDevice: %s", hipGetErrorString(e));
            if (rc[(size_t)i]) err[(size_t)i] = wv_last_error();
        });
        for (int i = 0; i < m->nl; i++)
            if (rc[(size_t)i]) return set_err(rc[(size_t)i], "%s", err[(size_t)i].c_str());
        return WV_OK;
    }
    for (int i0 = 0; i0 < m->nl; i0++) {
        const int i = m->sim && m->sim_rev ? m->nl - 1 - i0 : i0;
        MRank& R = *m->r[i];
        HIPCHK(hipSetDevice(R.dev));
        if (m->sim) HIPCHK(hipEventRecord(R.t0, R.s));
        int rc = fn(R, i);
        if (rc) return rc;
        if (m->sim) {
            HIPCHK(hipEventRecord(R.t1, R.s));
            HIPCHK(hipEventSynchronize(R.t1));
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, R.t0, R.t1));
            m->stage_ms[st][i] += ms;
        }
    }
    return WV_OK;
}

// one collective; with option sim timed as a whole (all local streams synced)
template <class Fn>
int run_xfer(wv_multi* m, Fn fn) {
    std::chrono::steady_clock::time_point t0;
    if (m->sim) t0 = std::chrono::steady_clock::now();
    int rc = fn();
    if (rc) return rc;
    if (m->sim) {
        for (auto& R : m->r) { HIPCHK(hipSetDevice(R->dev)); HIPCHK(hipStreamSynchronize(R->s)); }
        m->stage_ms[ST_XFER][0] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return WV_OK;
}

int gather(wv_multi* m, std::initializer_list<std::pair<DBuf MRank::*, DBuf MRank::*>> fields, std::initializer_list<size_t> bytes) {
    const int n = m->nl;
    std::vector<const void*> send;
    std::vector<void*> recv;
    for (auto& f : fields)
        for (int i = 0; i < n; i++) {
            send.push_back(((*m->r[i]).*(f.first)).p);
            recv.push_back(((*m->r[i]).*(f.second)).p);
        }
    std::vector<size_t> b(bytes);
    return run_xfer(m, [&] { return m->tr->all_gather((int)b.size(), send.data(), recv.data(), b.data()); });
}

int bcast(wv_multi* m, const std::vector<void*>& bufs, std::initializer_list<size_t> bytes, int root) {
    if (m->world == 1) return WV_OK;
    std::vector<size_t> b(bytes);
    return run_xfer(m, [&] { return m->tr->broadcast((int)b.size(), bufs.data(), b.data(), root); });
}

// the serial chain over a query list (sharded.py _replay_chain): rank r
// continues rank r-1's heap states, one broadcast per hop; every rank then
// writes the extracted rows into its merged results
int chain_list(wv_multi* m, int64_t nq, int64_t d, int k, DBuf MRank::*listp, int nlist, uint64_t* o_i0, float* o_d0,
               int32_t* o_n0) {
    const int W = m->world, n = m->nl;
    for (auto& Rp : m->r) {
        MRank& R = *Rp;
        HIPCHK(hipSetDevice(R.dev));
        for (int b = 0; b < 2; b++) {
            HIPCHK(R.ci[b].ensure((size_t)nlist * k * 8));
            HIPCHK(R.cd[b].ensure((size_t)nlist * k * 4));
            HIPCHK(R.cn[b].ensure((size_t)nlist * 4));
        }
    }
    for (int h = 0; h < W; h++) {
        const int cur = h & 1, prev = cur ^ 1;
        int rc = run_stage(m, ST_CHAIN, [&](MRank& R, int) -> int {
            if (R.rank != h) return WV_OK;
            m->n_chain++;
            return wv_index_replay_device(R.idx, R.qp, nq, d, k, (R.*listp).as<int32_t>(), nlist,
                                          h ? R.ci[prev].as<uint64_t>() : nullptr, h ? R.cd[prev].as<float>() : nullptr,
                                          h ? R.cn[prev].as<int32_t>() : nullptr, h == W - 1, R.ci[cur].as<uint64_t>(),
                                          R.cd[cur].as<float>(), R.cn[cur].as<int32_t>(), R.s);
        });
        if (rc) return rc;
        std::vector<void*> bufs;
        for (int f = 0; f < 3; f++)
            for (int i = 0; i < n; i++) {
                MRank& R = *m->r[i];
                bufs.push_back(f == 0 ? R.ci[cur].p : f == 1 ? R.cd[cur].p : R.cn[cur].p);
            }
        rc = bcast(m, bufs, {(size_t)nlist * k * 8, (size_t)nlist * k * 4, (size_t)nlist * 4}, h);
        if (rc) return rc;
    }
    const int last = (W - 1) & 1;
    return run_stage(m, ST_CHAIN, [&](MRank& R, int i) -> int {
        k_scatter_rows<<<(unsigned)nlist, 64, 0, R.s>>>((R.*listp).as<int32_t>(), nlist, k, R.ci[last].as<uint64_t>(),
                                                         R.cd[last].as<float>(), R.cn[last].as<int32_t>(),
                                                         i == 0 ? o_i0 : R.oi.as<uint64_t>(), i == 0 ? o_d0 : R.od.as<float>(),
                                                         i == 0 ? o_n0 : R.on.as<int32_t>());
        HIPCHK(hipGetLastError());
        return WV_OK;
    });
}

// every shard's work follows the caller's stream; queries go to each device once
int stage_queries(wv_multi* m, const float* q0, int64_t nq, int64_t d, hipStream_t cs) {
    MRank& H = *m->r[0];
    HIPCHK(hipSetDevice(H.dev));
    HIPCHK(hipEventRecord(m->e_call, cs));
    for (int i = 0; i < m->nl; i++) {
        MRank& R = *m->r[i];
        HIPCHK(hipSetDevice(R.dev));
        HIPCHK(hipStreamWaitEvent(R.s, m->e_call, 0));
        const size_t qb = (size_t)nq * d * 4;
        if (R.dev == H.dev) R.qp = q0;
        else {
            HIPCHK(R.q.ensure(qb));
            HIPCHK(hipMemcpyPeerAsync(R.q.p, R.dev, q0, H.dev, qb, R.s));
            R.qp = R.q.as<float>();
        }
    }
    return WV_OK;
}

// the caller's stream waits for every shard
int join_caller(wv_multi* m, hipStream_t cs) {
    MRank& H = *m->r[0];
    for (int i = 0; i < m->nl; i++) {
        MRank& R = *m->r[i];
        HIPCHK(hipSetDevice(R.dev));
        HIPCHK(hipEventRecord(R.e_out, R.s));
        HIPCHK(hipSetDevice(H.dev));
        HIPCHK(hipStreamWaitEvent(cs, R.e_out, 0));
    }
    return WV_OK;
}

int multi_search(wv_multi* m, const float* q0, int64_t nq, int64_t d, int k, uint64_t* o_i0, float* o_d0, int32_t* o_n0,
                 hipStream_t cs) {
    const int W = m->world, n = m->nl, k1 = k + 1;
    MRank& H = *m->r[0];
    int rc = stage_queries(m, q0, nq, d, cs);
    if (rc) return rc;
    for (int i = 0; i < n; i++) {
        MRank& R = *m->r[i];
        HIPCHK(hipSetDevice(R.dev));
        HIPCHK(R.topA.ensure((size_t)nq * k1 * 4));
        HIPCHK(R.eps.ensure((size_t)nq * 4));
        HIPCHK(R.gA.ensure((size_t)W * nq * k1 * 4));
        HIPCHK(R.gE.ensure((size_t)W * nq * 4));
        HIPCHK(R.ids.ensure((size_t)nq * k1 * 8));
        HIPCHK(R.dd.ensure((size_t)nq * k1 * 4));
        HIPCHK(R.cnt.ensure((size_t)nq * 4));
        HIPCHK(R.flg.ensure((size_t)nq * 4));
        HIPCHK(R.gi.ensure((size_t)W * nq * k1 * 8));
        HIPCHK(R.gd.ensure((size_t)W * nq * k1 * 4));
        HIPCHK(R.gc.ensure((size_t)W * nq * 4));
        HIPCHK(R.gf.ensure((size_t)W * nq * 4));
        if (i > 0) {
            HIPCHK(R.oi.ensure((size_t)nq * k * 8));
            HIPCHK(R.od.ensure((size_t)nq * k * 4));
            HIPCHK(R.on.ensure((size_t)nq * 4));
        }
        HIPCHK(R.of.ensure((size_t)nq * 4));
        HIPCHK(R.ql.ensure((size_t)nq * 4));
        HIPCHK(R.nl.ensure(16));
    }
    auto OI = [&](MRank& R, int i) { return i == 0 ? o_i0 : R.oi.as<uint64_t>(); };
    auto OD = [&](MRank& R, int i) { return i == 0 ? o_d0 : R.od.as<float>(); };
    auto ON = [&](MRank& R, int i) { return i == 0 ? o_n0 : R.on.as<int32_t>(); };

    // 1. phase 1
    rc = run_stage(m, ST_PHASE1, [&](MRank& R, int) -> int {
        R.off = false;
        int e = wv_index_shard_phase1(R.idx, R.qp, nq, d, k, R.topA.as<float>(), R.eps.as<float>(), R.s);
        if (e != WV_ERR_UNSUPPORTED) return e;
        // off the block-key path: no bound rows (the other ranks' cut stays valid)
        R.off = true;
        HIPCHK(hipSetDevice(R.dev));
        k_mfill_f32<<<(unsigned)((nq * k1 + 255) / 256), 256, 0, R.s>>>(R.topA.as<float>(), nq * k1, __builtin_inff());
        k_mfill_f32<<<(unsigned)((nq + 255) / 256), 256, 0, R.s>>>(R.eps.as<float>(), nq, 0.f);
        HIPCHK(hipGetLastError());
        return WV_OK;
    });
    if (rc) return rc;
    rc = gather(m, {{&MRank::topA, &MRank::gA}, {&MRank::eps, &MRank::gE}}, {(size_t)nq * k1 * 4, (size_t)nq * 4});
    if (rc) return rc;
    // 2. phase 2 (or the one-shot local search off the path)
    rc = run_stage(m, ST_PHASE2, [&](MRank& R, int) -> int {
        if (!R.off)
            return wv_index_shard_phase2(R.idx, W, nq, R.gA.as<float>(), R.gE.as<float>(), k, R.ids.as<uint64_t>(),
                                         R.dd.as<float>(), R.cnt.as<int32_t>(), R.flg.as<int32_t>(), R.s);
        return wv_index_search_device(R.idx, R.qp, nq, d, k, 1, R.ids.as<uint64_t>(), R.dd.as<float>(),
                                      R.cnt.as<int32_t>(), R.flg.as<int32_t>(), R.s);
    });
    if (rc) return rc;
    rc = gather(m, {{&MRank::ids, &MRank::gi}, {&MRank::dd, &MRank::gd}, {&MRank::cnt, &MRank::gc}, {&MRank::flg, &MRank::gf}},
                {(size_t)nq * k1 * 8, (size_t)nq * k1 * 4, (size_t)nq * 4, (size_t)nq * 4});
    if (rc) return rc;
    // 3. merge + the ascending flagged list
    rc = run_stage(m, ST_MERGE, [&](MRank& R, int i) -> int {
        int e = wv_merge_shards(R.dev, W, nq, k, R.gi.as<uint64_t>(), R.gd.as<float>(), R.gc.as<int32_t>(),
                                R.gf.as<int32_t>(), OI(R, i), OD(R, i), ON(R, i), R.of.as<int32_t>(), R.s);
        if (e) return e;
        k_list_ascending<<<1, 1024, 0, R.s>>>(R.of.as<int32_t>(), nullptr, (int)nq, R.ql.as<int32_t>(), R.nl.as<int32_t>());
        HIPCHK(hipGetLastError());
        if (i == 0) HIPCHK(hipMemcpyAsync(m->pin, R.nl.p, 4, hipMemcpyDeviceToHost, R.s));
        return WV_OK;
    });
    if (rc) return rc;
    HIPCHK(hipSetDevice(H.dev));
    HIPCHK(host_sync(m, H.s));  // host sync 1: the list length (equal on every rank)
    const int F = m->pin[0];
    m->last_flagged = F;
    m->n_flagged += F;
    if (F > 0 && k < 64) {
        // 4a. the parallel replay
        const int cap = m->rec_cap > 0 ? std::max(m->rec_cap, k) : std::max(256, 16 * k);
        rc = run_stage(m, ST_REPLAY, [&](MRank& R, int) -> int {
            HIPCHK(R.ri.ensure((size_t)F * cap * 8));
            HIPCHK(R.rd.ensure((size_t)F * cap * 4));
            HIPCHK(R.rn.ensure((size_t)F * 4));
            HIPCHK(R.gri.ensure((size_t)W * F * cap * 8));
            HIPCHK(R.grd.ensure((size_t)W * F * cap * 4));
            HIPCHK(R.grn.ensure((size_t)W * F * 4));
            if (R.rank == 0) {
                HIPCHK(R.ti.ensure((size_t)F * k * 8));
                HIPCHK(R.td.ensure((size_t)F * k * 4));
                HIPCHK(R.tn.ensure((size_t)F * 4));
                int e = wv_index_replay_device(R.idx, R.qp, nq, d, k, R.ql.as<int32_t>(), F, nullptr, nullptr, nullptr, 0,
                                               R.ti.as<uint64_t>(), R.td.as<float>(), R.tn.as<int32_t>(), R.s);
                if (e) return e;
                HIPCHK(hipSetDevice(R.dev));
                k_state_to_rec<<<(unsigned)F, 64, 0, R.s>>>(R.ti.as<uint64_t>(), R.td.as<float>(), R.tn.as<int32_t>(), F, k,
                                                             cap, R.ri.as<uint64_t>(), R.rd.as<float>(), R.rn.as<int32_t>());
                HIPCHK(hipGetLastError());
                return WV_OK;
            }
            HIPCHK(R.fki.ensure((size_t)F * k * 8));
            HIPCHK(R.fkd.ensure((size_t)F * k * 4));
            HIPCHK(R.fkn.ensure((size_t)F * 4));
            const size_t lds = (size_t)R.rank * k1 * 4;
            if (lds > 64 * 1024) return set_err(WV_ERR_UNSUPPORTED, "prefix bound: %d ranks x %d keys exceed LDS", R.rank, k1);
            k_prefix_bound<<<(unsigned)F, 256, lds, R.s>>>(R.rank, R.ql.as<int32_t>(), F, k, k1, nq, R.gd.as<float>(),
                                                           R.gc.as<int32_t>(), R.gf.as<int32_t>(), R.gA.as<float>(),
                                                           R.gE.as<float>(), R.fki.as<uint64_t>(), R.fkd.as<float>(),
                                                           R.fkn.as<int32_t>());
            HIPCHK(hipGetLastError());
            return wv_index_replay_record_device(R.idx, R.qp, nq, d, k, R.ql.as<int32_t>(), F, R.fki.as<uint64_t>(),
                                                 R.fkd.as<float>(), R.fkn.as<int32_t>(), cap, R.ri.as<uint64_t>(),
                                                 R.rd.as<float>(), R.rn.as<int32_t>(), R.s);
        });
        if (rc) return rc;
        rc = gather(m, {{&MRank::ri, &MRank::gri}, {&MRank::rd, &MRank::grd}, {&MRank::rn, &MRank::grn}},
                    {(size_t)F * cap * 8, (size_t)F * cap * 4, (size_t)F * 4});
        if (rc) return rc;
        rc = run_stage(m, ST_MERGE_REC, [&](MRank& R, int i) -> int {
            HIPCHK(R.sti.ensure((size_t)F * k * 8));
            HIPCHK(R.std_.ensure((size_t)F * k * 4));
            HIPCHK(R.fi.ensure((size_t)F * k * 8));
            HIPCHK(R.fd.ensure((size_t)F * k * 4));
            HIPCHK(R.fn.ensure((size_t)F * 4));
            HIPCHK(R.un.ensure((size_t)F * 4));
            HIPCHK(R.ul.ensure((size_t)F * 4));
            HIPCHK(R.nu.ensure(16));
            // rank 0's states: the first k entries of its gathered record rows
            HIPCHK(hipMemcpy2DAsync(R.sti.p, (size_t)k * 8, R.gri.p, (size_t)cap * 8, (size_t)k * 8, F,
                                    hipMemcpyDeviceToDevice, R.s));
            HIPCHK(hipMemcpy2DAsync(R.std_.p, (size_t)k * 4, R.grd.p, (size_t)cap * 4, (size_t)k * 4, F,
                                    hipMemcpyDeviceToDevice, R.s));
            int e = wv_heap_merge_records(R.dev, F, k, W, cap, R.sti.as<uint64_t>(), R.std_.as<float>(),
                                          R.grn.as<int32_t>(), R.gri.as<uint64_t>(), R.grd.as<float>(), R.grn.as<int32_t>(),
                                          R.fi.as<uint64_t>(), R.fd.as<float>(), R.fn.as<int32_t>(), R.un.as<int32_t>(), R.s);
            if (e) return e;
            HIPCHK(hipSetDevice(R.dev));
            k_scatter_rows<<<(unsigned)F, 64, 0, R.s>>>(R.ql.as<int32_t>(), F, k, R.fi.as<uint64_t>(), R.fd.as<float>(),
                                                        R.fn.as<int32_t>(), OI(R, i), OD(R, i), ON(R, i));
            k_list_ascending<<<1, 1024, 0, R.s>>>(R.un.as<int32_t>(), R.ql.as<int32_t>(), F, R.ul.as<int32_t>(),
                                                  R.nu.as<int32_t>());
            HIPCHK(hipGetLastError());
            if (i == 0) HIPCHK(hipMemcpyAsync(m->pin + 1, R.nu.p, 4, hipMemcpyDeviceToHost, R.s));
            return WV_OK;
        });
        if (rc) return rc;
        HIPCHK(hipSetDevice(H.dev));
        HIPCHK(host_sync(m, H.s));  // host sync 2: overflowed records (the same on every rank)
        const int U = m->pin[1];
        m->last_overflow = U;
        m->n_overflow += U;
        if (U > 0) {
            rc = chain_list(m, nq, d, k, &MRank::ul, U, o_i0, o_d0, o_n0);
            if (rc) return rc;
        }
    } else if (F > 0) {
        // 4b. k >= 64: the serial chain over the flags (states by query); the
        // last hop extracts into the merged results, which are broadcast
        for (auto& Rp : m->r) {
            MRank& R = *Rp;
            HIPCHK(hipSetDevice(R.dev));
            for (int b = 0; b < 2; b++) {
                HIPCHK(R.ci[b].ensure((size_t)nq * k * 8));
                HIPCHK(R.cd[b].ensure((size_t)nq * k * 4));
                HIPCHK(R.cn[b].ensure((size_t)nq * 4));
            }
        }
        for (int h = 0; h < W; h++) {
            const int cur = h & 1, prev = cur ^ 1;
            const bool last = h == W - 1;
            rc = run_stage(m, ST_CHAIN, [&](MRank& R, int i) -> int {
                if (R.rank != h) return WV_OK;
                m->n_chain++;
                return wv_index_replay_flags_device(
                    R.idx, R.qp, nq, d, k, R.of.as<int32_t>(), h ? R.ci[prev].as<uint64_t>() : nullptr,
                    h ? R.cd[prev].as<float>() : nullptr, h ? R.cn[prev].as<int32_t>() : nullptr, last ? 1 : 0,
                    last ? OI(R, i) : R.ci[cur].as<uint64_t>(), last ? OD(R, i) : R.cd[cur].as<float>(),
                    last ? ON(R, i) : R.cn[cur].as<int32_t>(), R.s);
            });
            if (rc) return rc;
            std::vector<void*> bufs;
            for (int f = 0; f < 3; f++)
                for (int i = 0; i < n; i++) {
                    MRank& R = *m->r[i];
                    bufs.push_back(f == 0 ? (last ? (void*)OI(R, i) : R.ci[cur].p)
                                   : f == 1 ? (last ? (void*)OD(R, i) : R.cd[cur].p)
                                            : (last ? (void*)ON(R, i) : R.cn[cur].p));
                }
            rc = bcast(m, bufs, {(size_t)nq * k * 8, (size_t)nq * k * 4, (size_t)nq * 4}, h);
            if (rc) return rc;
        }
    }
    return join_caller(m, cs);
}

// ---------------------------------------------------------------------------
// compressed searches: the R-heap of flat.searchByVectorQuantized (BQ, rq-8 /
// rq-1) or the worker heap of hnsw.flatSearch (trained PQ, SQ) across the
// shards in id order (sharded.py ShardedBQSearch / ShardedQuantSearch, DESIGN
// §4): every shard's compressed block minima in parallel; the R smallest
// minima of each shard all-gathered; shard 0 replays from empty heaps, shard
// r >= 1 from R copies of T_r recording its insertions; the records
// all-gathered and applied on shard 0's states (wv_heap_merge_records) = the
// serial chain's heaps (a record over its cap sends the chunk down that chain:
// one broadcast per hop); then the candidates each shard owns are rescored,
// the [world][nq][R] tiles all-gathered, and the rescoring heap runs on local
// shard 0 (the caller's outputs).
// ---------------------------------------------------------------------------
enum { MK_EXACT, MK_BQ, MK_QUANT };

int search_kind(const wv_index* i) {
    if (i->compression == WV_COMPRESSION_BQ) return MK_BQ;
    if (i->rq_bits || i->compression == WV_COMPRESSION_SQ || (i->compression == WV_COMPRESSION_PQ && i->pq_trained))
        return MK_QUANT;
    return MK_EXACT;  // uncompressed, or PQ before its codebook (the exact search, as one index runs it)
}

// the smallest of every rank's `v` (a batch size all ranks take): in-process
// worlds directly, otherwise one all-gather of 8 bytes per rank
int agree_min(wv_multi* m, const std::vector<int64_t>& local, int64_t* out) {
    int64_t v = INT64_MAX;
    for (int64_t x : local) v = std::min(v, x);
    if (m->world == 1 || m->nl == m->world) { *out = v; return WV_OK; }
    for (auto& Rp : m->r) {
        MRank& R = *Rp;
        HIPCHK(hipSetDevice(R.dev));
        HIPCHK(R.mb.ensure(8));
        HIPCHK(R.gmb.ensure((size_t)m->world * 8));
        HIPCHK(hipMemcpyAsync(R.mb.p, &v, 8, hipMemcpyHostToDevice, R.s));
    }
    int rc = gather(m, {{&MRank::mb, &MRank::gmb}}, {(size_t)8});
    if (rc) return rc;
    MRank& H = *m->r[0];
    std::vector<int64_t> all((size_t)m->world);
    HIPCHK(hipSetDevice(H.dev));
    HIPCHK(hipMemcpyAsync(all.data(), H.gmb.p, (size_t)m->world * 8, hipMemcpyDeviceToHost, H.s));
    for (auto& Rp : m->r) { HIPCHK(hipSetDevice(Rp->dev)); HIPCHK(hipStreamSynchronize(Rp->s)); }
    for (int64_t x : all) v = std::min(v, x);
    *out = v;
    return WV_OK;
}

int ensure_rank_iota(MRank& R, int64_t nq, hipStream_t s) {
    if (R.iota.bytes >= (size_t)nq * 4) return WV_OK;
    HIPCHK(R.iota.ensure((size_t)nq * 4));
    k_iota32<<<(unsigned)((R.iota.bytes / 4 + 255) / 256), 256, 0, s>>>(R.iota.as<int32_t>(), (int64_t)(R.iota.bytes / 4));
    HIPCHK(hipGetLastError());
    return WV_OK;
}

// the parallel R-heap over the shards for one chunk of nc queries (each shard's
// batch begun): bounds [nc][Rk] per shard (bounds_fn), replay states of shard 0
// (replay_fn), recorded replays of shards r >= 1 (record_fn), the merge.  On
// return *overflow = the chunk's queries whose record overflowed (0: fi / fd /
// fn hold the merged heaps extracted ascending on every shard).
template <class BoundsFn, class ReplayFn, class RecordFn>
int rheap_parallel(wv_multi* m, int64_t nc, int Rk, int cap, BoundsFn bounds_fn, ReplayFn replay_fn, RecordFn record_fn,
                   int* overflow) {
    const int W = m->world;
    int rc = run_stage(m, ST_PHASE2, [&](MRank& R, int) -> int {
        HIPCHK(R.bnd.ensure((size_t)nc * Rk * 4));
        HIPCHK(R.gbnd.ensure((size_t)W * nc * Rk * 4));
        return bounds_fn(R);
    });
    if (rc) return rc;
    rc = gather(m, {{&MRank::bnd, &MRank::gbnd}}, {(size_t)nc * Rk * 4});
    if (rc) return rc;
    rc = run_stage(m, ST_REPLAY, [&](MRank& R, int) -> int {
        HIPCHK(R.ri.ensure((size_t)nc * cap * 8));
        HIPCHK(R.rd.ensure((size_t)nc * cap * 4));
        HIPCHK(R.rn.ensure((size_t)nc * 4));
        HIPCHK(R.gri.ensure((size_t)W * nc * cap * 8));
        HIPCHK(R.grd.ensure((size_t)W * nc * cap * 4));
        HIPCHK(R.grn.ensure((size_t)W * nc * 4));
        if (R.rank == 0) {
            HIPCHK(R.ti.ensure((size_t)nc * Rk * 8));
            HIPCHK(R.td.ensure((size_t)nc * Rk * 4));
            HIPCHK(R.tn.ensure((size_t)nc * 4));
            int e = replay_fn(R);
            if (e) return e;
            HIPCHK(hipSetDevice(R.dev));
            k_state_to_rec<<<(unsigned)nc, 64, 0, R.s>>>(R.ti.as<uint64_t>(), R.td.as<float>(), R.tn.as<int32_t>(), (int)nc,
                                                          Rk, cap, R.ri.as<uint64_t>(), R.rd.as<float>(), R.rn.as<int32_t>());
            HIPCHK(hipGetLastError());
            return WV_OK;
        }
        HIPCHK(R.fki.ensure((size_t)nc * Rk * 8));
        HIPCHK(R.fkd.ensure((size_t)nc * Rk * 4));
        HIPCHK(R.fkn.ensure((size_t)nc * 4));
        const size_t lds = (size_t)R.rank * Rk * 4;
        if (lds > 160 * 1024) return set_err(WV_ERR_UNSUPPORTED, "prefix bound: %d ranks x %d minima exceed LDS", R.rank, Rk);
        HIPCHK(hipSetDevice(R.dev));
        if (lds > 64 * 1024)
            HIPCHK(hipFuncSetAttribute((const void*)k_prefix_bound, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        k_prefix_bound<<<(unsigned)nc, 256, lds, R.s>>>(R.rank, nullptr, (int)nc, Rk, Rk, nc, R.gbnd.as<float>(), nullptr,
                                                        nullptr, nullptr, nullptr, R.fki.as<uint64_t>(), R.fkd.as<float>(),
                                                        R.fkn.as<int32_t>());
        HIPCHK(hipGetLastError());
        return record_fn(R);
    });
    if (rc) return rc;
    rc = gather(m, {{&MRank::ri, &MRank::gri}, {&MRank::rd, &MRank::grd}, {&MRank::rn, &MRank::grn}},
                {(size_t)nc * cap * 8, (size_t)nc * cap * 4, (size_t)nc * 4});
    if (rc) return rc;
    rc = run_stage(m, ST_MERGE_REC, [&](MRank& R, int i) -> int {
        HIPCHK(R.sti.ensure((size_t)nc * Rk * 8));
        HIPCHK(R.std_.ensure((size_t)nc * Rk * 4));
        HIPCHK(R.fi.ensure((size_t)nc * Rk * 8));
        HIPCHK(R.fd.ensure((size_t)nc * Rk * 4));
        HIPCHK(R.fn.ensure((size_t)nc * 4));
        HIPCHK(R.un.ensure((size_t)nc * 4));
        HIPCHK(R.ul.ensure((size_t)nc * 4));
        HIPCHK(R.nu.ensure(16));
        HIPCHK(hipMemsetAsync(R.un.p, 0, (size_t)nc * 4, R.s));
        HIPCHK(hipMemcpy2DAsync(R.sti.p, (size_t)Rk * 8, R.gri.p, (size_t)cap * 8, (size_t)Rk * 8, nc,
                                hipMemcpyDeviceToDevice, R.s));
        HIPCHK(hipMemcpy2DAsync(R.std_.p, (size_t)Rk * 4, R.grd.p, (size_t)cap * 4, (size_t)Rk * 4, nc,
                                hipMemcpyDeviceToDevice, R.s));
        int e = wv_heap_merge_records(R.dev, (int)nc, Rk, W, cap, R.sti.as<uint64_t>(), R.std_.as<float>(),
                                      R.grn.as<int32_t>(), R.gri.as<uint64_t>(), R.grd.as<float>(), R.grn.as<int32_t>(),
                                      R.fi.as<uint64_t>(), R.fd.as<float>(), R.fn.as<int32_t>(), R.un.as<int32_t>(), R.s);
        if (e) return e;
        HIPCHK(hipSetDevice(R.dev));
        k_list_ascending<<<1, 1024, 0, R.s>>>(R.un.as<int32_t>(), nullptr, (int)nc, R.ul.as<int32_t>(), R.nu.as<int32_t>());
        HIPCHK(hipGetLastError());
        if (i == 0) HIPCHK(hipMemcpyAsync(m->pin + 1, R.nu.p, 4, hipMemcpyDeviceToHost, R.s));
        return WV_OK;
    });
    if (rc) return rc;
    MRank& H = *m->r[0];
    HIPCHK(hipSetDevice(H.dev));
    HIPCHK(host_sync(m, H.s));  // host sync: overflowed records (the same count on every rank)
    *overflow = m->pin[1];
    return WV_OK;
}

// the serial chain over the shards for one chunk (states [nc][Rk] by query): rank
// h continues rank h-1's heaps (hop_fn(R, in_i, in_d, in_n, last, out...)), one
// broadcast per hop; the last hop's output (pop order / extracted) ends in
// ci / cd / cn[(W - 1) & 1] of every shard
template <class HopFn>
int rheap_chain(wv_multi* m, int64_t nc, int Rk, HopFn hop_fn) {
    const int W = m->world, n = m->nl;
    for (auto& Rp : m->r) {
        MRank& R = *Rp;
        HIPCHK(hipSetDevice(R.dev));
        for (int b = 0; b < 2; b++) {
            HIPCHK(R.ci[b].ensure((size_t)nc * Rk * 8));
            HIPCHK(R.cd[b].ensure((size_t)nc * Rk * 4));
            HIPCHK(R.cn[b].ensure((size_t)nc * 4));
        }
    }
    for (int h = 0; h < W; h++) {
        const int cur = h & 1, prev = cur ^ 1;
        int rc = run_stage(m, ST_CHAIN, [&](MRank& R, int) -> int {
            if (R.rank != h) return WV_OK;
            m->n_chain++;
            return hop_fn(R, h ? R.ci[prev].as<uint64_t>() : nullptr, h ? R.cd[prev].as<float>() : nullptr,
                          h ? R.cn[prev].as<int32_t>() : nullptr, h == W - 1, R.ci[cur].as<uint64_t>(),
                          R.cd[cur].as<float>(), R.cn[cur].as<int32_t>());
        });
        if (rc) return rc;
        std::vector<void*> bufs;
        for (int f = 0; f < 3; f++)
            for (int i = 0; i < n; i++) {
                MRank& R = *m->r[i];
                bufs.push_back(f == 0 ? R.ci[cur].p : f == 1 ? R.cd[cur].p : R.cn[cur].p);
            }
        rc = bcast(m, bufs, {(size_t)nc * Rk * 8, (size_t)nc * Rk * 4, (size_t)nc * 4}, h);
        if (rc) return rc;
    }
    return WV_OK;
}

// candidates [nc][Rk] (global ids) -> each shard's exact distances of the ids it
// holds (rescore_fn), the tiles all-gathered into gEall [W][nc][Rk]
template <class RescoreFn>
int rescore_gather(wv_multi* m, int64_t nc, int Rk, RescoreFn rescore_fn) {
    const int W = m->world;
    int rc = run_stage(m, ST_MERGE, [&](MRank& R, int) -> int {
        HIPCHK(R.E.ensure((size_t)nc * Rk * 4));
        HIPCHK(R.gEall.ensure((size_t)W * nc * Rk * 4));
        HIPCHK(hipMemsetAsync(R.E.p, 0, (size_t)nc * Rk * 4, R.s));
        return rescore_fn(R);
    });
    if (rc) return rc;
    if (W == 1) {
        MRank& R = *m->r[0];
        HIPCHK(hipSetDevice(R.dev));
        HIPCHK(hipMemcpyAsync(R.gEall.p, R.E.p, (size_t)nc * Rk * 4, hipMemcpyDeviceToDevice, R.s));
        return WV_OK;
    }
    return gather(m, {{&MRank::E, &MRank::gEall}}, {(size_t)nc * Rk * 4});
}

// BQ (flat/index.go:460-532) over the shards, chunks of the batch that one
// block-minima group of every shard holds
int multi_search_bq(wv_multi* m, int64_t nq, int64_t d, int k, uint64_t* o_i0, float* o_d0, int32_t* o_n0) {
    const int W = m->world;
    std::vector<int64_t> mb;
    for (auto& R : m->r) mb.push_back(bq_max_batch(R->idx));
    int64_t chunk = 0;
    int rc = agree_min(m, mb, &chunk);
    if (rc) return rc;
    chunk = std::max<int64_t>(1, std::min(chunk, nq));
    for (int64_t c0 = 0; c0 < nq; c0 += chunk) {
        const int64_t nc = std::min(chunk, nq - c0);
        rc = run_stage(m, ST_PHASE1, [&](MRank& R, int) -> int {
            return wv_index_bq_begin(R.idx, R.qp + c0 * d, nc, d, k, R.s);
        });
        if (rc) return rc;
        const int Rk = m->r[0]->idx->bq_R;  // searchTimeRescore: max(rescore limit, k), equal on every shard
        bool chain = W == 1 || m->force_chain;
        // the candidates in pop order on every shard: the parallel form's
        // reversed merge (cand, fn) or the chain's last hop
        auto candv = [&](MRank& R) -> DBuf& { return chain ? R.ci[(W - 1) & 1] : R.cand; };
        auto cnv = [&](MRank& R) -> DBuf& { return chain ? R.cn[(W - 1) & 1] : R.fn; };
        if (!chain) {
            int ovf = 0;
            const int cap = m->rec_cap > 0 ? std::max(m->rec_cap, Rk) : 2 * Rk;
            rc = rheap_parallel(
                m, nc, Rk, cap,
                [&](MRank& R) { return wv_index_bq_bounds(R.idx, R.bnd.as<float>(), R.s); },
                [&](MRank& R) {
                    return wv_index_bq_replay(R.idx, nullptr, nullptr, nullptr, 0, R.ti.as<uint64_t>(), R.td.as<float>(),
                                              R.tn.as<int32_t>(), R.s);
                },
                [&](MRank& R) {
                    return wv_index_bq_replay_record(R.idx, R.fki.as<uint64_t>(), R.fkd.as<float>(), R.fkn.as<int32_t>(),
                                                     cap, R.ri.as<uint64_t>(), R.rd.as<float>(), R.rn.as<int32_t>(),
                                                     R.s);
                },
                &ovf);
            if (rc) return rc;
            m->last_overflow += ovf;
            m->n_overflow += ovf;
            if (ovf > 0) chain = true;
            else {
                rc = run_stage(m, ST_MERGE_REC, [&](MRank& R, int) -> int {
                    HIPCHK(R.cand.ensure((size_t)nc * Rk * 8));
                    k_rev_rows<<<(unsigned)nc, 64, 0, R.s>>>(R.fi.as<uint64_t>(), R.fn.as<int32_t>(), Rk,
                                                             R.cand.as<uint64_t>());
                    HIPCHK(hipGetLastError());
                    return WV_OK;
                });
                if (rc) return rc;
            }
        }
        if (chain) {
            rc = rheap_chain(m, nc, Rk, [&](MRank& R, const uint64_t* ii, const float* id, const int32_t* in, bool last,
                                            uint64_t* oi, float* od, int32_t* on) {
                return wv_index_bq_replay(R.idx, ii, id, in, last ? 1 : 0, oi, od, on, R.s);
            });
            if (rc) return rc;
        }
        rc = rescore_gather(m, nc, Rk, [&](MRank& R) {
            return wv_index_bq_rescore(R.idx, candv(R).as<uint64_t>(), cnv(R).as<int32_t>(), R.E.as<float>(), R.s);
        });
        if (rc) return rc;
        MRank& H = *m->r[0];
        HIPCHK(hipSetDevice(H.dev));
        rc = ensure_rank_iota(H, nc, H.s);
        if (rc) return rc;
        const size_t lds_f = (size_t)k * (sizeof(uint64_t) + sizeof(float)) + 16;
        if (lds_f > 64 * 1024)
            HIPCHK(hipFuncSetAttribute((const void*)k_bq_final, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_f));
        k_bq_final<<<(unsigned)nc, 64, lds_f, H.s>>>(candv(H).as<uint64_t>(), H.gEall.as<float>(),
                                                     cnv(H).as<int32_t>(), H.iota.as<int32_t>(), (int)nc, Rk, k, W,
                                                     m->id_stride, o_i0 + c0 * k, o_d0 + c0 * k, o_n0 + c0, 0);
        HIPCHK(hipGetLastError());
    }
    return WV_OK;
}

// trained PQ / SQ (hnsw/flat_search.go:28-141 + h.rescore) and flat rq-8 / rq-1
// (flat/index.go:460-532) over the shards: the worker heap of limit R across the
// shards, then the result heap / rescoring (wv_index_quant_*)
int multi_search_quant(wv_multi* m, int64_t nq, int64_t d, int k, uint64_t* o_i0, float* o_d0, int32_t* o_n0) {
    const int W = m->world;
    std::vector<int64_t> mb;
    for (auto& R : m->r) {
        int64_t v = 1;
        int rc = wv_index_quant_max_batch(R->idx, k, W, &v);
        if (rc) return rc;
        mb.push_back(v);
    }
    int64_t chunk = 0;
    int rc = agree_min(m, mb, &chunk);
    if (rc) return rc;
    chunk = std::max<int64_t>(1, std::min(chunk, nq));
    for (int64_t c0 = 0; c0 < nq; c0 += chunk) {
        const int64_t nc = std::min(chunk, nq - c0);
        int64_t info[64][4] = {};
        rc = run_stage(m, ST_PHASE1, [&](MRank& R, int i) -> int {
            int e = wv_index_quant_begin(R.idx, R.qp + c0 * d, nc, d, k, info[i], R.s);
            R.nblk = info[i][1];
            return e;
        });
        if (rc) return rc;
        const int Rk = (int)info[0][0], rescore = (int)info[0][2], form = (int)info[0][3];
        bool chain = W == 1 || m->force_chain;
        // the merged worker heap extracted ascending: the parallel form's merge
        // (fi, fd, fn) or the chain's last hop
        auto aiv = [&](MRank& R) -> DBuf& { return chain ? R.ci[(W - 1) & 1] : R.fi; };
        auto adv = [&](MRank& R) -> DBuf& { return chain ? R.cd[(W - 1) & 1] : R.fd; };
        auto anv = [&](MRank& R) -> DBuf& { return chain ? R.cn[(W - 1) & 1] : R.fn; };
        if (!chain) {
            int ovf = 0;
            const int cap = m->rec_cap > 0 ? std::max(m->rec_cap, Rk) : 2 * Rk + 64;
            rc = rheap_parallel(
                m, nc, Rk, cap,
                [&](MRank& R) -> int {
                    HIPCHK(R.bm.ensure((size_t)nc * R.nblk * 4));
                    int e = wv_index_quant_blockmin(R.idx, R.bm.as<float>(), R.s);
                    if (e) return e;
                    HIPCHK(hipSetDevice(R.dev));
                    k_smallest_r<<<(unsigned)nc, 256, 0, R.s>>>(R.bm.as<float>(), R.nblk, Rk, R.bnd.as<float>());
                    HIPCHK(hipGetLastError());
                    return WV_OK;
                },
                [&](MRank& R) {
                    return wv_index_quant_replay(R.idx, nullptr, nullptr, nullptr, 0, R.ti.as<uint64_t>(),
                                                 R.td.as<float>(), R.tn.as<int32_t>(), R.s);
                },
                [&](MRank& R) {
                    return wv_index_quant_replay_record(R.idx, R.fki.as<uint64_t>(), R.fkd.as<float>(),
                                                        R.fkn.as<int32_t>(), cap, R.ri.as<uint64_t>(), R.rd.as<float>(),
                                                        R.rn.as<int32_t>(), R.s);
                },
                &ovf);
            if (rc) return rc;
            m->last_overflow += ovf;
            m->n_overflow += ovf;
            chain = ovf > 0;
        }
        if (chain) {
            rc = rheap_chain(m, nc, Rk, [&](MRank& R, const uint64_t* ii, const float* id, const int32_t* in, bool last,
                                            uint64_t* oi, float* od, int32_t* on) {
                return wv_index_quant_replay(R.idx, ii, id, in, last ? 1 : 0, oi, od, on, R.s);
            });
            if (rc) return rc;
        }
        MRank& H = *m->r[0];
        if (!rescore) {
            HIPCHK(hipSetDevice(H.dev));
            rc = wv_index_quant_finish(H.idx, aiv(H).as<uint64_t>(), adv(H).as<float>(), anv(H).as<int32_t>(),
                                       o_i0 + c0 * k, o_d0 + c0 * k, o_n0 + c0, nullptr, nullptr, H.s);
            if (rc) return rc;
            continue;
        }
        rc = rescore_gather(m, nc, Rk, [&](MRank& R) -> int {
            HIPCHK(R.cand.ensure((size_t)nc * Rk * 8));
            HIPCHK(R.un.ensure((size_t)nc * 4));
            int e = wv_index_quant_finish(R.idx, aiv(R).as<uint64_t>(), adv(R).as<float>(), anv(R).as<int32_t>(),
                                          nullptr, nullptr, nullptr, R.cand.as<uint64_t>(), R.un.as<int32_t>(), R.s);
            if (e) return e;
            return wv_index_quant_rescore(R.idx, R.cand.as<uint64_t>(), R.un.as<int32_t>(), R.E.as<float>(), R.s);
        });
        if (rc) return rc;
        HIPCHK(hipSetDevice(H.dev));
        rc = ensure_rank_iota(H, nc, H.s);
        if (rc) return rc;
        if (form == 1) {  // searchByVectorQuantized's rescoring heap, candidates ascending
            const size_t lds_f = (size_t)k * (sizeof(uint64_t) + sizeof(float)) + 16;
            if (lds_f > 64 * 1024)
                HIPCHK(hipFuncSetAttribute((const void*)k_bq_final, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_f));
            k_bq_final<<<(unsigned)nc, 64, lds_f, H.s>>>(H.cand.as<uint64_t>(), H.gEall.as<float>(), H.un.as<int32_t>(),
                                                         H.iota.as<int32_t>(), (int)nc, Rk, k, W, m->id_stride,
                                                         o_i0 + c0 * k, o_d0 + c0 * k, o_n0 + c0, 1);
        } else {  // h.rescore
            const size_t lds_q = (size_t)(k + 1) * (sizeof(uint64_t) + sizeof(float)) + 16;
            if (lds_q > 64 * 1024)
                HIPCHK(hipFuncSetAttribute((const void*)k_pq_rescore_final, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds_q));
            k_pq_rescore_final<<<(unsigned)nc, 64, lds_q, H.s>>>(nullptr, H.gEall.as<float>(), H.un.as<int32_t>(),
                                                                 H.iota.as<int32_t>(), (int)nc, Rk, k, 0, o_i0 + c0 * k,
                                                                 o_d0 + c0 * k, o_n0 + c0, H.cand.as<uint64_t>(), W,
                                                                 m->id_stride);
        }
        HIPCHK(hipGetLastError());
    }
    return WV_OK;
}

// every search of the multi-shard index: the protocol of the shards' kind
int multi_dispatch(wv_multi* m, const float* q0, int64_t nq, int64_t d, int k, uint64_t* o_i0, float* o_d0, int32_t* o_n0,
                   hipStream_t cs) {
    const int kind = search_kind(m->r[0]->idx);
    for (auto& R : m->r)
        if (search_kind(R->idx) != kind)
            return set_err(WV_ERR_INVALID, "multi-shard index: shards differ in compression state (train every shard's "
                                           "quantizer: wv_multi_pq_fit / wv_multi_pq_set_centers)");
    if (m->sim) m->sim_n++;
    m->last_flagged = m->last_overflow = 0;
    m->host_wait_us = 0;
    const auto t_call = std::chrono::steady_clock::now();
    int rc;
    if (kind == MK_EXACT) rc = multi_search(m, q0, nq, d, k, o_i0, o_d0, o_n0, cs);
    else {
        rc = stage_queries(m, q0, nq, d, cs);
        if (!rc) rc = kind == MK_BQ ? multi_search_bq(m, nq, d, k, o_i0, o_d0, o_n0)
                                    : multi_search_quant(m, nq, d, k, o_i0, o_d0, o_n0);
        if (!rc) rc = join_caller(m, cs);
    }
    if (rc) return rc;
    m->host_total_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_call).count();
    m->n_search++;
    return WV_OK;
}

// A filtered search (the shard's allow list, shard_read.go:401-413 -> flat
// SearchByVector(..., allowList), :466): while the scope stands, every local
// shard reads present & allow (its part of the list) as its present bitmap, so
// every stage of every protocol -- keys, exact rows, replays, BQ / quantized
// minima -- scans only allowed rows.  Restored (and the batch state dropped)
// when the scope ends.
struct FilterScope {
    wv_multi* m = nullptr;
    ~FilterScope() { restore(); }
    void restore() {
        if (!m) return;
        for (auto& Rp : m->r) {
            MRank& R = *Rp;
            if (!R.saved_present) continue;
            hipSetDevice(R.dev);
            hipStreamSynchronize(R.s);  // no kernel of the search still reads the allow bitmap
            std::lock_guard<std::mutex> g(R.idx->mu);
            R.idx->present = R.saved_present;
            R.idx->npresent = R.saved_npresent;
            R.saved_present = nullptr;
            invalidate_batch(R.idx);
            note_mutation(R.idx);
        }
        m = nullptr;
    }
};

int filter_begin(wv_multi* m, FilterScope& fs, const uint64_t* allow, int64_t n_allow) {
    std::vector<std::vector<uint64_t>> part((size_t)m->nl);
    for (int64_t i = 0; i < n_allow; i++) {
        const int r = owner_rank(m, allow[i]) - m->rank0;
        if (r >= 0 && r < m->nl) part[(size_t)r].push_back(allow[i]);
    }
    fs.m = m;
    for (int i = 0; i < m->nl; i++) {
        MRank& R = *m->r[i];
        HIPCHK(hipSetDevice(R.dev));
        std::lock_guard<std::mutex> g(R.idx->mu);
        const uint32_t* valid = nullptr;
        int64_t nv = 0;
        int rc = shard_filter_bitmap(R.idx, R.s, part[(size_t)i].data(), (int64_t)part[(size_t)i].size(), &valid, &nv);
        if (rc) return rc;
        R.saved_present = R.idx->present;
        R.saved_npresent = R.idx->npresent;
        R.idx->present = const_cast<uint32_t*>(valid);
        R.idx->npresent = nv;
        invalidate_batch(R.idx);
        note_mutation(R.idx);
    }
    return WV_OK;
}

}  // namespace

extern "C" int wv_rccl_unique_id(void* out, int64_t cap) {
    if (!out || cap < (int64_t)sizeof(ncclUniqueId)) return set_err(WV_ERR_INVALID, "unique id buffer < %d bytes", (int)sizeof(ncclUniqueId));
    const RcclApi& a = rccl();
    if (!a.ok) return set_err(WV_ERR_UNSUPPORTED, "%s", a.err.c_str());
    ncclUniqueId id;
    RCCLCHK(a.GetUniqueId(&id));
    memcpy(out, &id, sizeof(id));
    return WV_OK;
}

extern "C" void wv_multi_destroy(wv_multi* m) {
    if (!m) return;
    for (auto& R : m->r) {
        hipSetDevice(R->dev);
        if (R->s) hipStreamSynchronize(R->s);
    }
    m->pool.reset();
    m->tr.reset();
    for (auto& R : m->r) {
        hipSetDevice(R->dev);
        if (R->idx) wv_index_destroy(R->idx);
        for (hipEvent_t e : {R->e_out, R->e_in, R->t0, R->t1})
            if (e) hipEventDestroy(e);
        if (R->s) hipStreamDestroy(R->s);
    }
    if (!m->r.empty()) hipSetDevice(m->r[0]->dev);
    if (m->e_call) hipEventDestroy(m->e_call);
    if (m->pin) hipHostFree(m->pin);
    delete m;
}

extern "C" int wv_multi_create(const wv_multi_config* cfg, wv_multi** out) {
    if (!cfg || !out) return set_err(WV_ERR_INVALID, "invalid config: nil");
    *out = nullptr;
    if (cfg->world < 1 || cfg->n_local < 1 || cfg->rank0 < 0 || cfg->rank0 + cfg->n_local > cfg->world || !cfg->devices)
        return set_err(WV_ERR_INVALID, "invalid multi config: world %d, rank0 %d, n_local %d", cfg->world, cfg->rank0,
                       cfg->n_local);
    if (cfg->n_local > 64) return set_err(WV_ERR_INVALID, "at most 64 shards per process");
    if (cfg->index.compression < WV_COMPRESSION_NONE || cfg->index.compression > WV_COMPRESSION_SQ)
        return set_err(WV_ERR_INVALID, "unknown compression %d", cfg->index.compression);
    if (cfg->transport != WV_TRANSPORT_LOCAL && cfg->transport != WV_TRANSPORT_RCCL &&
        cfg->transport != WV_TRANSPORT_HOST)
        return set_err(WV_ERR_INVALID, "unknown transport %d", cfg->transport);
    if (cfg->transport == WV_TRANSPORT_HOST && (cfg->n_local != 1 || !cfg->host_allgather || !cfg->host_broadcast))
        return set_err(WV_ERR_INVALID, "host transport: one local shard and both callbacks");
    if (cfg->transport == WV_TRANSPORT_LOCAL && cfg->n_local != cfg->world)
        return set_err(WV_ERR_INVALID, "local transport: every rank must be a local shard");
    if (cfg->transport == WV_TRANSPORT_RCCL && cfg->n_local != cfg->world && !cfg->unique_id)
        return set_err(WV_ERR_INVALID, "RCCL transport over processes needs the unique id of rank 0");
    if (cfg->world > 1 && cfg->id_stride == 0) return set_err(WV_ERR_INVALID, "id_stride must be positive");
    wv_multi* m = new wv_multi();
    m->world = cfg->world;
    m->rank0 = cfg->rank0;
    m->nl = cfg->n_local;
    m->kind = cfg->transport;
    m->id_stride = cfg->id_stride;
    auto fail = [&](int rc) { wv_multi_destroy(m); return rc; };
    for (int i = 0; i < m->nl; i++) {
        auto R = std::make_unique<MRank>();
        R->dev = cfg->devices[i];
        R->rank = cfg->rank0 + i;
        wv_config c = cfg->index;
        c.device = R->dev;
        c.id_base = (uint64_t)R->rank * cfg->id_stride;
        int rc = wv_index_create(&c, &R->idx);
        // the protocol drives the shards on its own streams: no per-call graph capture
        if (!rc) rc = wv_index_set_option(R->idx, "graph", 0);
        if (rc) { m->r.push_back(std::move(R)); return fail(rc); }
        hipError_t e = hipSetDevice(R->dev);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&R->s, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&R->e_out, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&R->e_in, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreate(&R->t0);
        if (e == hipSuccess) e = hipEventCreate(&R->t1);
        m->r.push_back(std::move(R));
        if (e != hipSuccess) return fail(set_err(WV_ERR_HIP, "multi shard %d: %s", i, hipGetErrorString(e)));
    }
    hipError_t e = hipSetDevice(m->r[0]->dev);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&m->e_call, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc((void**)&m->pin, 64, hipHostMallocDefault);
    if (e != hipSuccess) return fail(set_err(WV_ERR_HIP, "multi: %s", hipGetErrorString(e)));
    std::unique_ptr<Transport> tr;
    int rc;
    if (cfg->transport == WV_TRANSPORT_LOCAL) {
        auto t = std::make_unique<LocalTransport>();
        for (auto& R : m->r) { t->dev.push_back(R->dev); t->s.push_back(R->s); }
        rc = t->init();
        tr = std::move(t);
    } else if (cfg->transport == WV_TRANSPORT_HOST) {
        auto t = std::make_unique<HostTransport>();
        for (auto& R : m->r) { t->dev.push_back(R->dev); t->s.push_back(R->s); }
        t->world = m->world;
        t->rank = m->rank0;
        t->ag = cfg->host_allgather;
        t->bc = cfg->host_broadcast;
        t->user = cfg->host_user;
        rc = WV_OK;
        tr = std::move(t);
    } else {
        auto t = std::make_unique<RcclTransport>();
        for (auto& R : m->r) { t->dev.push_back(R->dev); t->s.push_back(R->s); }
        rc = t->init(m->world, m->rank0, cfg->unique_id);
        tr = std::move(t);
    }
    m->tr = std::move(tr);
    if (rc) return fail(rc);
    if (m->nl > 1) m->pool = std::make_unique<StagePool>(m->nl);
    *out = m;
    return WV_OK;
}

extern "C" wv_index* wv_multi_shard(wv_multi* m, int32_t local) {
    if (!m || local < 0 || local >= m->nl) return nullptr;
    return m->r[local]->idx;
}

extern "C" int wv_multi_set_option(wv_multi* m, const char* key, int64_t value) {
    if (!m || !key) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(m->mu);
    if (std::string(key) == "sim") {  // (re)starts the averaging
        m->sim = value ? 1 : 0;
        m->sim_n = 0;
        memset(m->stage_ms, 0, sizeof(m->stage_ms));
        return WV_OK;
    }
    if (std::string(key) == "host_threads") {  // 0: one host thread issues every shard's stages
        if (!value) m->pool.reset();
        else if (!m->pool && m->nl > 1) m->pool = std::make_unique<StagePool>(m->nl);
        return WV_OK;
    }
    if (std::string(key) == "sim_rev") {
        m->sim_rev = value ? 1 : 0;
        return WV_OK;
    }
    if (std::string(key) == "chain") {
        m->force_chain = value ? 1 : 0;
        return WV_OK;
    }
    if (std::string(key) == "rec_cap") {
        if (value < 0 || value > (1 << 20)) return set_err(WV_ERR_INVALID, "rec_cap out of range");
        m->rec_cap = (int)value;
        return WV_OK;
    }
    for (auto& R : m->r) {
        int rc = wv_index_set_option(R->idx, key, value);
        if (rc) return rc;
    }
    return WV_OK;
}

extern "C" int wv_multi_add_batch(wv_multi* m, const uint64_t* ids, const float* vecs, int64_t n, int64_t d) {
    if (!m) return set_err(WV_ERR_INVALID, "nil index");
    if (n <= 0) return set_err(WV_ERR_INSERT, "insertBatch called with empty lists");
    if (!ids || !vecs || d <= 0) return set_err(WV_ERR_INVALID, "nil buffer");
    std::lock_guard<std::mutex> g(m->mu);
    std::vector<std::vector<int64_t>> rows(m->nl);
    for (int64_t i = 0; i < n; i++) {
        const int r = owner_rank(m, ids[i]) - m->rank0;
        if (r < 0 || r >= m->nl)
            return set_err(WV_ERR_INVALID, "id %llu belongs to rank %d, not a shard of this process",
                           (unsigned long long)ids[i], r + m->rank0);
        rows[r].push_back(i);
    }
    // ValidateBeforeInsert on every receiving shard first: a failed call inserts nothing
    for (int r = 0; r < m->nl; r++)
        if (!rows[r].empty()) {
            int rc = wv_index_validate_before_insert(m->r[r]->idx, d);
            if (rc) return rc;
        }
    std::vector<uint64_t> si;
    std::vector<float> sv;
    for (int r = 0; r < m->nl; r++) {
        if (rows[r].empty()) continue;
        si.resize(rows[r].size());
        sv.resize(rows[r].size() * d);
        for (size_t j = 0; j < rows[r].size(); j++) {
            si[j] = ids[rows[r][j]];
            memcpy(&sv[j * d], vecs + rows[r][j] * d, (size_t)d * 4);
        }
        int rc = wv_index_add_batch(m->r[r]->idx, si.data(), sv.data(), (int64_t)si.size(), d);
        if (rc) return rc;
    }
    return WV_OK;
}

extern "C" int wv_multi_search_device(wv_multi* m, const float* d_queries, int64_t nq, int64_t d, int32_t k,
                                      uint64_t* d_ids, float* d_dists, int32_t* d_counts, void* stream) {
    if (!m) return set_err(WV_ERR_INVALID, "nil index");
    if (k <= 0) return set_err(WV_ERR_INVALID, "k must be positive (reference heap Top() on empty queue)");
    if (nq < 0 || (nq > 0 && (!d_queries || !d_ids || !d_dists || !d_counts))) return set_err(WV_ERR_INVALID, "nil buffer");
    if (nq == 0) return WV_OK;
    std::lock_guard<std::mutex> g(m->mu);
    int rc = multi_dispatch(m, d_queries, nq, d, k, d_ids, d_dists, d_counts, (hipStream_t)stream);
    if (rc) return rc;
    if (!stream) {
        HIPCHK(hipSetDevice(m->r[0]->dev));
        HIPCHK(hipStreamSynchronize(nullptr));
    }
    return WV_OK;
}

namespace {
int check_allow(const uint64_t* allow_ids, int64_t n_allow, int32_t allow_mode) {
    if (allow_mode != 0 && allow_mode != 1) return set_err(WV_ERR_INVALID, "allow mode %d", allow_mode);
    if (allow_mode == 1 && (n_allow < 0 || (n_allow > 0 && !allow_ids))) return set_err(WV_ERR_INVALID, "nil allow ids");
    return WV_OK;
}

// one batch from host buffers (m->mu held); allow_mode 1: under the allow list
int multi_host_batch(wv_multi* m, const float* queries, int64_t nq, int64_t d, int32_t k, const uint64_t* allow_ids,
                     int64_t n_allow, int32_t allow_mode, uint64_t* out_ids, float* out_dists, int32_t* out_counts) {
    if (allow_mode == 1 && n_allow == 0) {  // flat/index.go:590-594: an empty allow list finds nothing
        for (int64_t q = 0; q < nq; q++) out_counts[q] = 0;
        return WV_OK;
    }
    MRank& H = *m->r[0];
    HIPCHK(hipSetDevice(H.dev));
    DBuf q, oi, od, on;
    HIPCHK(q.ensure((size_t)nq * d * 4));
    HIPCHK(oi.ensure((size_t)nq * k * 8));
    HIPCHK(od.ensure((size_t)nq * k * 4));
    HIPCHK(on.ensure((size_t)nq * 4));
    HIPCHK(hipMemcpyAsync(q.p, queries, (size_t)nq * d * 4, hipMemcpyHostToDevice, H.s));
    FilterScope fs;
    int rc = allow_mode == 1 ? filter_begin(m, fs, allow_ids, n_allow) : WV_OK;
    if (!rc) rc = multi_dispatch(m, q.as<float>(), nq, d, k, oi.as<uint64_t>(), od.as<float>(), on.as<int32_t>(), H.s);
    if (rc) {
        for (auto& R : m->r) { hipSetDevice(R->dev); hipStreamSynchronize(R->s); }
        return rc;
    }
    HIPCHK(hipSetDevice(H.dev));
    HIPCHK(hipMemcpyAsync(out_ids, oi.p, (size_t)nq * k * 8, hipMemcpyDeviceToHost, H.s));
    HIPCHK(hipMemcpyAsync(out_dists, od.p, (size_t)nq * k * 4, hipMemcpyDeviceToHost, H.s));
    HIPCHK(hipMemcpyAsync(out_counts, on.p, (size_t)nq * 4, hipMemcpyDeviceToHost, H.s));
    HIPCHK(hipStreamSynchronize(H.s));
    return WV_OK;
}
}  // namespace

extern "C" int wv_multi_search_device_allow(wv_multi* m, const float* d_queries, int64_t nq, int64_t d, int32_t k,
                                            const uint64_t* allow_ids, int64_t n_allow, int32_t allow_mode,
                                            uint64_t* d_ids, float* d_dists, int32_t* d_counts, void* stream) {
    if (!m) return set_err(WV_ERR_INVALID, "nil index");
    if (k <= 0) return set_err(WV_ERR_INVALID, "k must be positive (reference heap Top() on empty queue)");
    if (nq < 0 || (nq > 0 && (!d_queries || !d_ids || !d_dists || !d_counts))) return set_err(WV_ERR_INVALID, "nil buffer");
    int rc = check_allow(allow_ids, n_allow, allow_mode);
    if (rc) return rc;
    if (nq == 0) return WV_OK;
    std::lock_guard<std::mutex> g(m->mu);
    hipStream_t cs = (hipStream_t)stream;
    HIPCHK(hipSetDevice(m->r[0]->dev));
    if (allow_mode == 1 && n_allow == 0) {
        HIPCHK(hipMemsetAsync(d_counts, 0, (size_t)nq * 4, cs));
    } else {
        FilterScope fs;
        rc = allow_mode == 1 ? filter_begin(m, fs, allow_ids, n_allow) : WV_OK;
        if (!rc) rc = multi_dispatch(m, d_queries, nq, d, k, d_ids, d_dists, d_counts, cs);
        if (rc) return rc;
    }
    if (!stream) {
        HIPCHK(hipSetDevice(m->r[0]->dev));
        HIPCHK(hipStreamSynchronize(nullptr));
    }
    return WV_OK;
}

extern "C" int wv_multi_search_by_vector_batch(wv_multi* m, const float* queries, int64_t nq, int64_t d, int32_t k,
                                               uint64_t* out_ids, float* out_dists, int32_t* out_counts) {
    return wv_multi_search_by_vector_batch_allow(m, queries, nq, d, k, nullptr, 0, 0, out_ids, out_dists, out_counts);
}

extern "C" int wv_multi_search_by_vector_batch_allow(wv_multi* m, const float* queries, int64_t nq, int64_t d, int32_t k,
                                                     const uint64_t* allow_ids, int64_t n_allow, int32_t allow_mode,
                                                     uint64_t* out_ids, float* out_dists, int32_t* out_counts) {
    if (!m) return set_err(WV_ERR_INVALID, "nil index");
    if (k <= 0) return set_err(WV_ERR_INVALID, "k must be positive (reference heap Top() on empty queue)");
    int rc = check_allow(allow_ids, n_allow, allow_mode);
    if (rc) return rc;
    if (nq <= 0) return WV_OK;
    if (!queries || !out_ids || !out_dists || !out_counts || d <= 0) return set_err(WV_ERR_INVALID, "nil buffer");
    std::lock_guard<std::mutex> g(m->mu);
    return multi_host_batch(m, queries, nq, d, k, allow_ids, n_allow, allow_mode, out_ids, out_dists, out_counts);
}

extern "C" int wv_multi_search_by_vector_batch_multi_allow(wv_multi* m, const float* queries, int64_t nq, int64_t d,
                                                           int32_t k, const uint64_t* allow_ids,
                                                           const int64_t* allow_offsets, const int32_t* allow_modes,
                                                           uint64_t* out_ids, float* out_dists, int32_t* out_counts) {
    if (!m) return set_err(WV_ERR_INVALID, "nil index");
    if (k <= 0) return set_err(WV_ERR_INVALID, "k must be positive (reference heap Top() on empty queue)");
    if (nq <= 0) return WV_OK;
    if (!queries || !out_ids || !out_dists || !out_counts || !allow_offsets || !allow_modes || d <= 0)
        return set_err(WV_ERR_INVALID, "nil buffer");
    for (int64_t q = 0; q < nq; q++) {
        if (allow_modes[q] != 0 && allow_modes[q] != 1) return set_err(WV_ERR_INVALID, "allow mode %d", allow_modes[q]);
        if (allow_offsets[q] < 0 || allow_offsets[q + 1] < allow_offsets[q])
            return set_err(WV_ERR_INVALID, "allow offsets not ascending at %lld", (long long)q);
        if (allow_modes[q] == 1 && allow_offsets[q + 1] > allow_offsets[q] && !allow_ids)
            return set_err(WV_ERR_INVALID, "nil allow ids");
    }
    std::lock_guard<std::mutex> g(m->mu);
    // the queries grouped by identical list (every process groups the same
    // queries and lists the same way: the map orders its keys), one filtered
    // search over every shard per group
    std::map<std::pair<int, std::string>, std::vector<int64_t>> groups;
    for (int64_t q = 0; q < nq; q++) {
        std::string key;
        if (allow_modes[q] == 1)
            key.assign(reinterpret_cast<const char*>(allow_ids + allow_offsets[q]),
                       (size_t)(allow_offsets[q + 1] - allow_offsets[q]) * sizeof(uint64_t));
        groups[{allow_modes[q], key}].push_back(q);
    }
    std::vector<float> qb;
    std::vector<uint64_t> oi;
    std::vector<float> od;
    std::vector<int32_t> on;
    for (auto& gq : groups) {
        const std::vector<int64_t>& qs = gq.second;
        const int64_t n = (int64_t)qs.size(), q0 = qs[0];
        qb.resize((size_t)n * d);
        oi.assign((size_t)n * k, 0);
        od.assign((size_t)n * k, 0.f);
        on.assign((size_t)n, 0);
        for (int64_t i = 0; i < n; i++) memcpy(&qb[(size_t)i * d], queries + qs[(size_t)i] * d, (size_t)d * 4);
        int rc = multi_host_batch(m, qb.data(), n, d, k, allow_modes[q0] ? allow_ids + allow_offsets[q0] : nullptr,
                                  allow_offsets[q0 + 1] - allow_offsets[q0], allow_modes[q0], oi.data(), od.data(),
                                  on.data());
        if (rc) return rc;
        for (int64_t i = 0; i < n; i++) {
            const int64_t q = qs[(size_t)i];
            memcpy(out_ids + q * k, &oi[(size_t)i * k], (size_t)k * 8);
            memcpy(out_dists + q * k, &od[(size_t)i * k], (size_t)k * 4);
            out_counts[q] = on[(size_t)i];
        }
    }
    return WV_OK;
}

// flat.SearchByVectorDistance (flat/index.go:699-761) over every shard: one
// search with totalLimit = 100, then the results up to the target distance
// (as wv_index_search_by_vector_distance); the per-shard calls of
// shard_read.go:439 merged by distance (index.go:2067-2071) give the same rows
extern "C" int wv_multi_search_by_vector_distance(wv_multi* m, const float* query, int64_t d, float target,
                                                  int64_t max_limit, const uint64_t* allow_ids, int64_t n_allow,
                                                  int32_t allow_mode, uint64_t* out_ids, float* out_dists,
                                                  int32_t* out_count) {
    (void)max_limit;
    if (!m) return set_err(WV_ERR_INVALID, "nil index");
    if (!query || !out_ids || !out_dists || !out_count || d <= 0) return set_err(WV_ERR_INVALID, "nil buffer");
    int rc = check_allow(allow_ids, n_allow, allow_mode);
    if (rc) return rc;
    const int total_limit = 100;
    std::vector<uint64_t> ids(total_limit);
    std::vector<float> dd(total_limit);
    int32_t n = 0;
    {
        std::lock_guard<std::mutex> g(m->mu);
        rc = multi_host_batch(m, query, 1, d, total_limit, allow_ids, n_allow, allow_mode, ids.data(), dd.data(), &n);
    }
    if (rc) return rc;
    int cnt = 0;
    for (int i = 0; i < n && i < total_limit; i++) {
        const double diff = std::fabs((double)dd[i] - (double)target);
        if (dd[i] <= target || diff <= 1e-6) { out_ids[cnt] = ids[i]; out_dists[cnt] = dd[i]; cnt++; }
        else break;
    }
    *out_count = cnt;
    return WV_OK;
}

// ProductQuantizer.Fit for every shard (product_quantization.go:378-424): the
// single index trains on its first trainingLimit present rows in id order; the
// multi-shard index gathers those rows from the shards in rank order (one
// process holding every rank) or finds them all on rank 0 (a world over
// processes), trains there, and installs the codebook on every shard
// (NewProductQuantizerWithEncoders, :193-203).
extern "C" int wv_multi_pq_fit(wv_multi* m, uint64_t seed) {
    if (!m) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(m->mu);
    for (auto& R : m->r)
        if (R->idx->compression != WV_COMPRESSION_PQ) return set_err(WV_ERR_INVALID, "pq_fit: index is not PQ-compressed");
    MRank& H = *m->r[0];
    wv_index* hi = H.idx;
    const int64_t L = hi->pq_training_limit > 0 ? hi->pq_training_limit : INT64_MAX;
    const int64_t nfl = (int64_t)hi->pq_m * hi->pq_ks * (hi->dims > 0 && hi->pq_m > 0 ? hi->dims / hi->pq_m : 0);
    int rc = WV_OK;
    if (m->nl == m->world) {
        // every rank here: the first L present rows of the shards in rank order
        std::vector<std::pair<int, std::vector<uint32_t>>> take;
        int64_t n = 0;
        for (int i = 0; i < m->nl && n < L; i++) {
            wv_index* x = m->r[i]->idx;
            std::lock_guard<std::mutex> gi(x->mu);
            std::vector<uint32_t> sl;
            for (int64_t s = 0; s < x->hiwater && n < L; s++)
                if (x->h_present[s]) { sl.push_back((uint32_t)s); n++; }
            take.push_back({i, std::move(sl)});
        }
        if (hi->dims == 0) return set_err(WV_ERR_INVALID, "pq: dimensions not set yet");
        for (auto& t : take)
            if (m->r[t.first]->idx->dims != hi->dims && !t.second.empty())
                return set_err(WV_ERR_INVALID, "pq_fit: shards differ in dimensions");
        HIPCHK(hipSetDevice(H.dev));
        DBuf T;
        const int64_t ld = hi->dpad;
        HIPCHK(T.ensure((size_t)std::max<int64_t>(n, 1) * ld * 4));
        int64_t row = 0;
        for (auto& t : take) {
            MRank& R = *m->r[t.first];
            const std::vector<uint32_t>& sl = t.second;
            for (size_t a = 0; a < sl.size();) {  // runs of consecutive slots: one copy each
                size_t b = a + 1;
                while (b < sl.size() && sl[b] == sl[b - 1] + 1) b++;
                const size_t bytes = (b - a) * (size_t)ld * 4;
                const float* src = R.idx->X + (int64_t)sl[a] * ld;
                if (R.dev == H.dev) HIPCHK(hipMemcpyAsync(T.as<float>() + row * ld, src, bytes, hipMemcpyDeviceToDevice, H.s));
                else HIPCHK(hipMemcpyPeerAsync(T.as<float>() + row * ld, H.dev, src, R.dev, bytes, H.s));
                row += (int64_t)(b - a);
                a = b;
            }
        }
        HIPCHK(hipStreamSynchronize(H.s));
        std::lock_guard<std::mutex> gh(hi->mu);
        rc = pq_fit_rows(hi, T.as<float>(), n, seed);
        hipStreamSynchronize(hi->stream);
        if (rc) return rc;
    } else {
        // a world over processes: the training rows must all lie on rank 0,
        // which trains (every rank learns whether it could, so none waits alone)
        std::vector<int64_t> st(1, 1);
        std::string err;
        if (H.rank == 0) {
            {
                std::lock_guard<std::mutex> gh(hi->mu);
                if (hi->pq_training_limit <= 0 || hi->npresent < hi->pq_training_limit) st[0] = 0;
            }
            if (st[0] && wv_index_pq_fit(hi, seed) != WV_OK) {
                err = wv_last_error();
                st[0] = 0;
            }
        }
        int64_t all_ok = 0;
        rc = agree_min(m, st, &all_ok);
        if (rc) return rc;
        if (!all_ok)
            return H.rank == 0 && !err.empty()
                       ? set_err(WV_ERR_UNSUPPORTED, "pq_fit on rank 0: %s", err.c_str())
                       : set_err(WV_ERR_UNSUPPORTED, "pq_fit: rank 0 could not train on the first trainingLimit rows "
                                                     "(they span the processes' shards: fit one index and install "
                                                     "its codebook with wv_multi_pq_set_centers)");
    }
    // the codebook from rank 0 to every shard
    std::vector<float> hc((size_t)nfl);
    for (auto& Rp : m->r) {
        MRank& R = *Rp;
        HIPCHK(hipSetDevice(R.dev));
        HIPCHK(R.bm.ensure((size_t)nfl * 4));
        if (R.rank == 0) {
            rc = wv_index_pq_centers(R.idx, hc.data(), nfl);
            if (rc) return rc;
            HIPCHK(hipMemcpy(R.bm.p, hc.data(), (size_t)nfl * 4, hipMemcpyHostToDevice));
        }
    }
    std::vector<void*> bufs;
    for (auto& Rp : m->r) bufs.push_back(Rp->bm.p);
    rc = bcast(m, bufs, {(size_t)nfl * 4}, 0);
    if (rc) return rc;
    for (auto& Rp : m->r) {
        MRank& R = *Rp;
        if (R.rank == 0) continue;
        HIPCHK(hipSetDevice(R.dev));
        HIPCHK(hipStreamSynchronize(R.s));
        HIPCHK(hipMemcpy(hc.data(), R.bm.p, (size_t)nfl * 4, hipMemcpyDeviceToHost));
        rc = wv_index_pq_set_centers(R.idx, hc.data(), nfl);
        if (rc) return rc;
    }
    return WV_OK;
}

// NewProductQuantizerWithEncoders on every shard (a codebook trained elsewhere)
extern "C" int wv_multi_pq_set_centers(wv_multi* m, const float* centers, int64_t n_floats) {
    if (!m || !centers) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(m->mu);
    for (auto& R : m->r) {
        int rc = wv_index_pq_set_centers(R->idx, centers, n_floats);
        if (rc) return rc;
    }
    return WV_OK;
}

extern "C" int wv_multi_stats(wv_multi* m, int64_t* out, int32_t n) {
    if (!m || !out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(m->mu);
    const int64_t v[] = {m->n_search, m->n_flagged, m->n_overflow, m->n_chain, m->last_flagged, m->last_overflow,
                         m->world, m->rank0, m->nl, m->kind, (int64_t)m->host_total_us, (int64_t)m->host_wait_us};
    for (int i = 0; i < n && i < (int)(sizeof(v) / sizeof(v[0])); i++) out[i] = v[i];
    return WV_OK;
}

extern "C" int wv_multi_stage_ms(wv_multi* m, double* out, int32_t n_local_cap) {
    if (!m || !out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(m->mu);
    const int nl = std::min(m->nl, (int)n_local_cap);
    const double div = m->sim_n > 0 ? (double)m->sim_n : 1.0;
    for (int s = 0; s < ST_N; s++)
        for (int i = 0; i < nl; i++) out[s * nl + i] = m->stage_ms[s][i] / div;
    return WV_OK;
}
