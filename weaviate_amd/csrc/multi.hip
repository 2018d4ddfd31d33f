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
__global__ __launch_bounds__(256) void k_prefix_bound(int r, const int32_t* __restrict__ ql, int F, int k, int k1, int64_t nq,
                                                      const float* __restrict__ gd, const int32_t* __restrict__ gc,
                                                      const int32_t* __restrict__ gf, const float* __restrict__ gA,
                                                      const float* __restrict__ gE, uint64_t* __restrict__ oi,
                                                      float* __restrict__ od, int32_t* __restrict__ on) {
    extern __shared__ float pbv[];
    __shared__ float slot;
    const int li = blockIdx.x;
    if (li >= F) return;
    const int64_t q = ql[li];
    const int n = r * k1;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int rr = i / k1, j = i - rr * k1;
        const int64_t row = (int64_t)rr * nq + q;
        pbv[i] = (j < gc[row] && gf[row] == 0) ? gd[row * k1 + j] : __builtin_inff();
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

}  // namespace

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
};

struct wv_multi {
    std::mutex mu;
    int world = 1, rank0 = 0, nl = 1, kind = WV_TRANSPORT_LOCAL;
    uint64_t id_stride = 0;
    std::vector<std::unique_ptr<MRank>> r;
    std::unique_ptr<Transport> tr;
    hipEvent_t e_call = nullptr;
    int32_t* pin = nullptr;  // pinned host words: flagged count, overflow count
    int sim = 0;
    int rec_cap = 0;  // option rec_cap (tests): replay record capacity, 0 = max(256, 16 k)
    double stage_ms[ST_N][64] = {};  // option sim: stage times summed over sim_n searches
    int64_t sim_n = 0;
    int64_t n_search = 0, n_flagged = 0, n_overflow = 0, n_chain = 0, last_flagged = 0, last_overflow = 0;
};

namespace {

int owner_rank(const wv_multi* m, uint64_t id) {
    const uint64_t r = m->id_stride ? id / m->id_stride : 0;
    return (int)std::min<uint64_t>(r, (uint64_t)(m->world - 1));
}

// issue one stage on every local shard; with option sim every shard's part is
// timed alone (HIP events, then a sync before the next shard)
template <class Fn>
int run_stage(wv_multi* m, int st, Fn fn) {
    for (int i = 0; i < m->nl; i++) {
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

int multi_search(wv_multi* m, const float* q0, int64_t nq, int64_t d, int k, uint64_t* o_i0, float* o_d0, int32_t* o_n0,
                 hipStream_t cs) {
    const int W = m->world, n = m->nl, k1 = k + 1;
    if (m->sim) m->sim_n++;
    m->last_flagged = m->last_overflow = 0;
    // every shard's work follows the caller's stream; queries go to each device once
    MRank& H = *m->r[0];
    HIPCHK(hipSetDevice(H.dev));
    HIPCHK(hipEventRecord(m->e_call, cs));
    for (int i = 0; i < n; i++) {
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
    int rc = run_stage(m, ST_PHASE1, [&](MRank& R, int) -> int {
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
    HIPCHK(hipStreamSynchronize(H.s));  // host sync 1: the list length (equal on every rank)
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
        HIPCHK(hipStreamSynchronize(H.s));  // host sync 2: overflowed records (the same on every rank)
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
    // the caller's stream waits for every shard
    for (int i = 0; i < n; i++) {
        MRank& R = *m->r[i];
        HIPCHK(hipSetDevice(R.dev));
        HIPCHK(hipEventRecord(R.e_out, R.s));
        HIPCHK(hipSetDevice(H.dev));
        HIPCHK(hipStreamWaitEvent(cs, R.e_out, 0));
    }
    m->n_search++;
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
    if (cfg->index.compression != WV_COMPRESSION_NONE)
        return set_err(WV_ERR_UNSUPPORTED, "multi-shard index: exact (uncompressed) search only");
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
    int rc = multi_search(m, d_queries, nq, d, k, d_ids, d_dists, d_counts, (hipStream_t)stream);
    if (rc) return rc;
    if (!stream) {
        HIPCHK(hipSetDevice(m->r[0]->dev));
        HIPCHK(hipStreamSynchronize(nullptr));
    }
    return WV_OK;
}

extern "C" int wv_multi_search_by_vector_batch(wv_multi* m, const float* queries, int64_t nq, int64_t d, int32_t k,
                                               uint64_t* out_ids, float* out_dists, int32_t* out_counts) {
    if (!m) return set_err(WV_ERR_INVALID, "nil index");
    if (k <= 0) return set_err(WV_ERR_INVALID, "k must be positive (reference heap Top() on empty queue)");
    if (nq <= 0) return WV_OK;
    if (!queries || !out_ids || !out_dists || !out_counts || d <= 0) return set_err(WV_ERR_INVALID, "nil buffer");
    std::lock_guard<std::mutex> g(m->mu);
    MRank& H = *m->r[0];
    HIPCHK(hipSetDevice(H.dev));
    DBuf q, oi, od, on;
    HIPCHK(q.ensure((size_t)nq * d * 4));
    HIPCHK(oi.ensure((size_t)nq * k * 8));
    HIPCHK(od.ensure((size_t)nq * k * 4));
    HIPCHK(on.ensure((size_t)nq * 4));
    HIPCHK(hipMemcpyAsync(q.p, queries, (size_t)nq * d * 4, hipMemcpyHostToDevice, H.s));
    int rc = multi_search(m, q.as<float>(), nq, d, k, oi.as<uint64_t>(), od.as<float>(), on.as<int32_t>(), H.s);
    if (rc) { hipStreamSynchronize(H.s); return rc; }
    HIPCHK(hipSetDevice(H.dev));
    HIPCHK(hipMemcpyAsync(out_ids, oi.p, (size_t)nq * k * 8, hipMemcpyDeviceToHost, H.s));
    HIPCHK(hipMemcpyAsync(out_dists, od.p, (size_t)nq * k * 4, hipMemcpyDeviceToHost, H.s));
    HIPCHK(hipMemcpyAsync(out_counts, on.p, (size_t)nq * 4, hipMemcpyDeviceToHost, H.s));
    HIPCHK(hipStreamSynchronize(H.s));
    return WV_OK;
}

extern "C" int wv_multi_stats(wv_multi* m, int64_t* out, int32_t n) {
    if (!m || !out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(m->mu);
    const int64_t v[] = {m->n_search, m->n_flagged, m->n_overflow, m->n_chain, m->last_flagged, m->last_overflow,
                         m->world, m->rank0, m->nl, m->kind};
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
