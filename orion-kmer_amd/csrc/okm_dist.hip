// okm_dist.hip — the multi-GPU merge inside the library:
// key-range owners, RCCL over xGMI, hand-written pack/unpack kernels.
//
// Reads shard by record across GPUs (count.rs:23-38 is per record), every
// rank counts its shard into its own sorted table (okm_count), and ONE
// exchange turns the P local tables into the global one (the single DashMap of
// count.rs:48, drained and sorted at count.rs:106-119):
//
//   1. 2^16-bin histogram of the top key bits of the local SORTED table: one
//      binary search per bin start (k_bin_bounds), no pass over the keys;
//   2. ncclAllReduce of the histogram; the host cuts it into count-balanced
//      contiguous key ranges, one per rank (okm_owner_bounds: value-range
//      ownership, so the global table is the concatenation of the owners'
//      ranges in rank order and needs no final merge; canonical k-mers are
//      skewed ~7:5:3:1 by first base, so equal-width ranges would not balance);
//   3. the local table splits at the range starts (binary search again) and
//      moves with grouped ncclSend/ncclRecv: keys as u64, counts as ONE byte
//      (k_pack_counts: the low byte; a count > 255 also travels as an escape
//      (position, value) that overwrites the byte on arrival, k_apply_escapes):
//      9 B per pair on a point-to-point xGMI link instead of 16;
//   4. the owner adds every rank's slice — each one sorted — without copying
//      (okm_add_sorted_pairs_device) and counts them as key-range items split
//      out of every slice by binary search: counts add, the fetch_add of
//      count.rs:31-34.
//
// RCCL is loaded at run time (dlopen), so the library still loads where no
// RCCL is installed; only the okm_comm_* calls then fail, with OKM_E_COMM.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "okm_dev_common.h"
#include "okm_hip_try.h"

namespace okm {

// ---------------------------------------------------------------------------
// RCCL entry points (dlopen)
// ---------------------------------------------------------------------------
struct Rccl {
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
    bool ok = false;
    std::string why;
};

static Rccl load_rccl() {
    Rccl r;
    std::vector<std::string> names;
    if (const char *e = getenv("OKM_RCCL_LIB")) names.push_back(e);
    names.push_back("librccl.so.1");
    names.push_back("librccl.so");
    names.push_back("/opt/rocm/lib/librccl.so.1");
    void *h = nullptr;
    for (auto &n : names)
        if ((h = dlopen(n.c_str(), RTLD_NOW | RTLD_LOCAL))) break;
    if (!h) {
        r.why = std::string("RCCL not found (librccl.so.1): ") + (dlerror() ? dlerror() : "");
        return r;
    }
    bool all = true;
    auto sym = [&](auto &fn, const char *name) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
        if (!fn) {
            all = false;
            r.why += std::string(" missing ") + name;
        }
    };
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRank, "ncclCommInitRank");
    sym(r.CommInitAll, "ncclCommInitAll");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.AllReduce, "ncclAllReduce");
    sym(r.AllGather, "ncclAllGather");
    sym(r.Send, "ncclSend");
    sym(r.Recv, "ncclRecv");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.GetErrorString, "ncclGetErrorString");
    r.ok = all;
    return r;
}

static Rccl &rccl() {
    static Rccl r = load_rccl();
    return r;
}

#define NCCL_TRY(expr)                                                                                   \
    do {                                                                                                 \
        ncclResult_t r_ = (expr);                                                                        \
        if (r_ != ncclSuccess)                                                                           \
            return fail(OKM_E_COMM, std::string(#expr) + ": " + rccl().GetErrorString(r_));              \
    } while (0)

// ---------------------------------------------------------------------------
// Owner split (host): count-balanced contiguous bin ranges
// ---------------------------------------------------------------------------

// bounds[0] = 0 <= bounds[1] <= ... <= bounds[world] = nbins; rank r owns bins
// [bounds[r], bounds[r+1]).  Cut r lands just past the bin where the running
// total first reaches r/world of the whole (dist.py's numpy restatement is
// checked against this in the CPU tests).
static void owner_bounds(const uint64_t *hist, uint32_t nbins, int world, uint32_t *bounds) {
    std::vector<double> cum(nbins);
    double run = 0;
    for (uint32_t b = 0; b < nbins; ++b) cum[b] = (run += (double)hist[b]);
    const double total = nbins ? cum[nbins - 1] : 0.0;
    bounds[0] = 0;
    for (int r = 1; r < world; ++r) {
        const double target = total * r / world;
        const uint32_t b = (uint32_t)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin()) + 1;
        bounds[r] = std::max(bounds[r - 1], std::min(b, nbins));
    }
    bounds[world] = nbins;
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------

__global__ void k_hist_from_starts(const ull *__restrict__ starts, uint32_t nb, ull *__restrict__ hist) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) hist[b] = starts[b + 1] - starts[b];
}

__device__ __forceinline__ uint32_t dest_of(const ull *cut, uint32_t P, uint64_t i) {
    uint32_t lo = 0, hi = P;  // last r with cut[r] <= i
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cut[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

// Low byte of every count (4 per thread: two 16-B loads, one 4-B store, so
// a wave's loads and stores are contiguous); WRITE=false counts the escapes
// (count > 255) per destination, WRITE=true also writes them, grouped by
// destination: (position in the destination's run, count).
constexpr int kPackPer = 4;
constexpr uint64_t kPackBlock = 256 * kPackPer;  // counts per workgroup

template <bool WRITE>
__global__ __launch_bounds__(256) void k_pack_counts(const uint64_t *__restrict__ counts, uint64_t n,
                                                     const ull *__restrict__ cut, uint32_t P, uint8_t *__restrict__ low,
                                                     ull *__restrict__ esc_cnt, ull *__restrict__ esc_cur,
                                                     uint64_t *__restrict__ esc, uint64_t skip0, uint64_t skip1) {
    // [skip0, skip1): this rank's own slice when the owner borrows it (never sent)
    const uint64_t b0 = (uint64_t)blockIdx.x * kPackBlock;
    if (b0 >= skip0 && b0 + kPackBlock <= skip1) return;  // block-uniform
    const uint64_t i0 = b0 + (uint64_t)threadIdx.x * kPackPer;
    if (i0 >= n) return;
    uint64_t c[kPackPer] = {0, 0, 0, 0};
    if (i0 + kPackPer <= n) {
        const ulonglong2 *p = reinterpret_cast<const ulonglong2 *>(counts + i0);
        const ulonglong2 v0 = p[0], v1 = p[1];
        c[0] = v0.x, c[1] = v0.y, c[2] = v1.x, c[3] = v1.y;
    } else {
        for (int j = 0; j < kPackPer && i0 + j < n; ++j) c[j] = counts[i0 + j];
    }
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < kPackPer; ++j) {
        const uint64_t i = i0 + j;
        if (i >= skip0 && i < skip1) c[j] = 0;
        if (c[j] > 255) {
            const uint32_t d = dest_of(cut, P, i);
            if (WRITE) {
                const ull s = atomicAdd(&esc_cur[d], 1ull);
                esc[2 * s] = i - cut[d];
                esc[2 * s + 1] = c[j];
            } else {
                atomicAdd(&esc_cnt[d], 1ull);
            }
        }
        word |= (uint32_t)(c[j] & 0xFFu) << (8 * j);
    }
    if (WRITE) return;  // the bytes are written by the counting pass
    if (i0 + kPackPer <= n)
        *reinterpret_cast<uint32_t *>(low + i0) = word;
    else
        for (int j = 0; j < kPackPer && i0 + j < n; ++j) low[i0 + j] = (uint8_t)(word >> (8 * j));
}

__global__ __launch_bounds__(256) void k_widen_counts(const uint8_t *__restrict__ low, uint64_t n,
                                                      uint64_t *__restrict__ counts) {
    const uint64_t i0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * kPackPer;
    if (i0 >= n) return;
    if (i0 + kPackPer <= n) {
        const uint32_t w = *reinterpret_cast<const uint32_t *>(low + i0);
        ulonglong2 *p = reinterpret_cast<ulonglong2 *>(counts + i0);
        p[0] = make_ulonglong2(w & 0xFFu, (w >> 8) & 0xFFu);
        p[1] = make_ulonglong2((w >> 16) & 0xFFu, w >> 24);
    } else {
        for (int j = 0; j < kPackPer && i0 + j < n; ++j) counts[i0 + j] = low[i0 + j];
    }
}

// Escapes received from rank s sit at esc[2 * reoff[s] ..]: counts[roff[s] + pos] = value.
__global__ void k_apply_escapes(const uint64_t *__restrict__ esc, uint64_t nesc, const ull *__restrict__ reoff,
                                const ull *__restrict__ roff, uint32_t P, uint64_t *__restrict__ counts) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nesc) return;
    const uint32_t s = dest_of(reoff, P, j);
    counts[roff[s] + esc[2 * j]] = esc[2 * j + 1];
}

}  // namespace okm

using namespace okm;

// ---------------------------------------------------------------------------
// Communicator
// ---------------------------------------------------------------------------
namespace {
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    okm_status ensure(size_t bytes) {
        if (bytes <= cap) return OKM_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 8, 4096);
        HIP_TRY(hipMalloc(&p, want));
        cap = want;
        return OKM_OK;
    }
    template <typename T> T *as() const { return static_cast<T *>(p); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};
}  // namespace

struct okm_comm {
    int device = 0, rank = 0, size = 1;
    ncclComm_t nc = nullptr;
    hipStream_t stream = nullptr;
    DevBuf starts, hist, hsum, cut, sizes, gsizes, low, esc_cnt, esc_cur, esc, rk, rlow, rc, resc, offs;
    ull *hpin = nullptr;  // pinned landing area for the small readbacks
    size_t hpin_cap = 0;
    double last_ms[4] = {0, 0, 0, 0};  // plan, exchange, unpack, merge (host wall, last okm_merge_owned)
};

namespace {
okm_status ensure_hpin(okm_comm *m, size_t words) {
    if (words <= m->hpin_cap) return OKM_OK;
    if (m->hpin) (void)hipHostFree(m->hpin);
    m->hpin = nullptr;
    m->hpin_cap = 0;
    HIP_TRY(hipHostMalloc(&m->hpin, words * sizeof(ull), hipHostMallocDefault));
    m->hpin_cap = words;
    return OKM_OK;
}

okm_status comm_finish_init(okm_comm *m) {
    HIP_TRY(hipSetDevice(m->device));
    HIP_TRY(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
    return OKM_OK;
}

double ms_since(const std::chrono::steady_clock::time_point &t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace

extern "C" {

okm_status okm_owner_bounds(const uint64_t *hist, uint32_t nbins, int world, uint32_t *bounds) {
    if (!bounds || world < 1 || (nbins && !hist)) return fail(OKM_E_ARG, "okm_owner_bounds: bad arguments");
    owner_bounds(hist, nbins, world, bounds);
    return OKM_OK;
}

okm_status okm_comm_unique_id(uint8_t *id) {
    if (!id) return fail(OKM_E_ARG, "okm_comm_unique_id: null id");
    if (!rccl().ok) return fail(OKM_E_COMM, rccl().why);
    ncclUniqueId u;
    NCCL_TRY(rccl().GetUniqueId(&u));
    static_assert(sizeof(u) == OKM_COMM_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, sizeof(u));
    return OKM_OK;
}

okm_status okm_comm_init_rank(okm_comm **out, int nranks, int rank, const uint8_t *id, int device) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(OKM_E_ARG, "okm_comm_init_rank: bad arguments");
    *out = nullptr;
    if (!rccl().ok) return fail(OKM_E_COMM, rccl().why);
    HIP_TRY(hipSetDevice(device));
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    okm_comm *m = new okm_comm();
    m->device = device;
    m->rank = rank;
    m->size = nranks;
    ncclResult_t r = rccl().CommInitRank(&m->nc, nranks, u, rank);
    if (r != ncclSuccess) {
        delete m;
        return fail(OKM_E_COMM, std::string("ncclCommInitRank: ") + rccl().GetErrorString(r));
    }
    okm_status st = comm_finish_init(m);
    if (st != OKM_OK) {
        okm_comm_destroy(m);
        return st;
    }
    *out = m;
    return OKM_OK;
}

okm_status okm_comm_init_all(okm_comm **out, int n, const int *devices) {
    if (!out || n < 1) return fail(OKM_E_ARG, "okm_comm_init_all: bad arguments");
    if (!rccl().ok) return fail(OKM_E_COMM, rccl().why);
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) devs[i] = devices ? devices[i] : i;
    std::vector<ncclComm_t> ncs(n);
    NCCL_TRY(rccl().CommInitAll(ncs.data(), n, devs.data()));
    for (int i = 0; i < n; ++i) {
        okm_comm *m = new okm_comm();
        m->device = devs[i];
        m->rank = i;
        m->size = n;
        m->nc = ncs[i];
        out[i] = m;
        okm_status st = comm_finish_init(m);
        if (st != OKM_OK) {
            for (int j = 0; j <= i; ++j) okm_comm_destroy(out[j]);
            for (int j = i + 1; j < n; ++j) (void)rccl().CommDestroy(ncs[j]);
            return st;
        }
    }
    return OKM_OK;
}

void okm_comm_destroy(okm_comm *m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    if (m->nc) (void)rccl().CommDestroy(m->nc);
    for (DevBuf *b : {&m->starts, &m->hist, &m->hsum, &m->cut, &m->sizes, &m->gsizes, &m->low, &m->esc_cnt,
                      &m->esc_cur, &m->esc, &m->rk, &m->rlow, &m->rc, &m->resc, &m->offs})
        b->release();
    if (m->hpin) (void)hipHostFree(m->hpin);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

int okm_comm_rank(const okm_comm *m) { return m ? m->rank : -1; }
int okm_comm_size(const okm_comm *m) { return m ? m->size : 0; }

okm_status okm_comm_last_times(const okm_comm *m, double *ms4) {
    if (!m || !ms4) return fail(OKM_E_ARG, "null argument");
    for (int i = 0; i < 4; ++i) ms4[i] = m->last_ms[i];
    return OKM_OK;
}

okm_status okm_merge_owned(okm_ctx *local, okm_comm *m, okm_ctx *owner, uint64_t *n_owned) {
    if (!local || !m || !owner) return fail(OKM_E_ARG, "okm_merge_owned: null argument");
    if (ctx_device(local) != m->device || ctx_device(owner) != m->device)
        return fail(OKM_E_ARG, "okm_merge_owned: local, owner and communicator must share one device");
    // owner == local is allowed (and cheapest: one context, one device pool):
    // the local table is only read until the exchange has completed
    if (ctx_is_wide(local) || ctx_is_wide(owner) || ctx_k(local) != ctx_k(owner))
        return fail(OKM_E_ARG, "okm_merge_owned: k must match and be <= 32");
    const auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipSetDevice(m->device));
    const uint64_t *dk = nullptr, *dc = nullptr;
    uint64_t n = 0;
    OKM_TRY(okm_result_device(local, &dk, &dc, &n));  // counts the local shard if needed (synchronous)
    const bool set = ctx_is_set(local) || ctx_is_set(owner);
    const uint32_t P = (uint32_t)m->size, me = (uint32_t)m->rank;
    const uint32_t k = ctx_k(local);
    const uint32_t bits = std::min<uint32_t>(16, 2 * k);
    const uint32_t nb = 1u << bits, shift = 2 * k - bits;
    hipStream_t s = m->stream;

    // 1-2. histogram of the sorted table's top bits, summed over ranks
    OKM_TRY(m->starts.ensure((nb + 1) * sizeof(ull)));
    OKM_TRY(m->hist.ensure(nb * sizeof(ull)));
    OKM_TRY(m->hsum.ensure(nb * sizeof(ull)));
    launch_bin_bounds(s, dk, n, shift, nb, m->starts.as<ull>(), false);
    hipLaunchKernelGGL(k_hist_from_starts, dim3((nb + 255) / 256), dim3(256), 0, s, m->starts.as<ull>(), nb,
                       m->hist.as<ull>());
    HIP_TRY(hipGetLastError());
    NCCL_TRY(rccl().AllReduce(m->hist.p, m->hsum.p, nb, ncclUint64, ncclSum, m->nc, s));
    OKM_TRY(ensure_hpin(m, 2 * (size_t)nb + 1 + 8 * (size_t)P * P + 64));
    ull *h_sum = m->hpin, *h_starts = m->hpin + nb;
    HIP_TRY(hipMemcpyAsync(h_sum, m->hsum.p, nb * sizeof(ull), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(h_starts, m->starts.p, (nb + 1) * sizeof(ull), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<uint32_t> bounds(P + 1);
    owner_bounds(reinterpret_cast<const uint64_t *>(h_sum), nb, (int)P, bounds.data());
    std::vector<ull> cut(P + 1);
    for (uint32_t r = 0; r <= P; ++r) cut[r] = bounds[r] >= nb ? n : h_starts[bounds[r]];
    cut[0] = 0;
    cut[P] = n;

    // 3. sizes (and escape counts) of every pair of ranks
    OKM_TRY(m->cut.ensure((P + 1) * sizeof(ull)));
    OKM_TRY(m->sizes.ensure(2 * P * sizeof(ull)));
    OKM_TRY(m->gsizes.ensure(2 * (size_t)P * P * sizeof(ull)));
    OKM_TRY(m->esc_cnt.ensure(P * sizeof(ull)));
    OKM_TRY(m->esc_cur.ensure((P + 1) * sizeof(ull)));
    HIP_TRY(hipMemcpyAsync(m->cut.p, cut.data(), (P + 1) * sizeof(ull), hipMemcpyHostToDevice, s));
    std::vector<ull> hs(2 * P, 0);
    for (uint32_t r = 0; r < P; ++r) hs[r] = cut[r + 1] - cut[r];
    HIP_TRY(hipMemcpyAsync(m->sizes.p, hs.data(), P * sizeof(ull), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(m->sizes.as<ull>() + P, 0, P * sizeof(ull), s));
    const uint64_t pblocks = (n + kPackBlock - 1) / kPackBlock;
    // This rank's own slice never crosses RCCL when the owner is another
    // context: the owner borrows it straight from the local table (it stays
    // unchanged until okm_count(owner) returns below).  owner == local
    // receives it through a self send/recv, since okm_reset(owner) releases it.
    const bool self_borrow = owner != local;
    const uint64_t skip0 = self_borrow ? cut[me] : 0, skip1 = self_borrow ? cut[me + 1] : 0;
    if (!set) {
        OKM_TRY(m->low.ensure(std::max<uint64_t>(n, 16)));
        if (pblocks)
            hipLaunchKernelGGL(k_pack_counts<false>, dim3((uint32_t)pblocks), dim3(256), 0, s, dc, n, m->cut.as<ull>(),
                               P, m->low.as<uint8_t>(), m->sizes.as<ull>() + P, nullptr, nullptr, skip0, skip1);
        HIP_TRY(hipGetLastError());
    }
    NCCL_TRY(rccl().AllGather(m->sizes.p, m->gsizes.p, 2 * P, ncclUint64, m->nc, s));
    ull *h_g = m->hpin + 2 * (size_t)nb + 1;
    HIP_TRY(hipMemcpyAsync(h_g, m->gsizes.p, 2 * (size_t)P * P * sizeof(ull), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<ull> ss(P), rs(P), es(P), er(P), roff(P + 1, 0), reoff(P + 1, 0), eoff(P + 1, 0);
    for (uint32_t r = 0; r < P; ++r) {
        ss[r] = h_g[(size_t)me * 2 * P + r];
        es[r] = h_g[(size_t)me * 2 * P + P + r];
        rs[r] = h_g[(size_t)r * 2 * P + me];
        er[r] = h_g[(size_t)r * 2 * P + P + me];
        roff[r + 1] = roff[r] + rs[r];
        reoff[r + 1] = reoff[r] + er[r];
        eoff[r + 1] = eoff[r] + es[r];
    }
    const uint64_t self_n = ss[me];
    if (self_borrow) {
        for (uint32_t r = me + 1; r <= P; ++r) roff[r] -= rs[me], reoff[r] -= er[me];
        rs[me] = er[me] = 0;
        ss[me] = es[me] = 0;
    }
    const uint64_t nrecv = roff[P], nresc = reoff[P], nesc = eoff[P];
    if (!set && nesc) {  // escapes grouped by destination
        OKM_TRY(m->esc.ensure(2 * nesc * sizeof(uint64_t)));
        HIP_TRY(hipMemcpyAsync(m->esc_cur.p, eoff.data(), P * sizeof(ull), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_pack_counts<true>, dim3((uint32_t)pblocks), dim3(256), 0, s, dc, n, m->cut.as<ull>(), P,
                           m->low.as<uint8_t>(), nullptr, m->esc_cur.as<ull>(), m->esc.as<uint64_t>(), skip0, skip1);
        HIP_TRY(hipGetLastError());
    }
    const double t_plan = ms_since(t0);

    // 4. move the slices: keys as u64, counts as bytes (+ escapes)
    OKM_TRY(m->rk.ensure(std::max<uint64_t>(nrecv, 1) * sizeof(uint64_t)));
    if (!set) {
        OKM_TRY(m->rlow.ensure(std::max<uint64_t>(nrecv, 16)));
        OKM_TRY(m->rc.ensure(std::max<uint64_t>(nrecv, 1) * sizeof(uint64_t)));
        OKM_TRY(m->resc.ensure(std::max<uint64_t>(2 * nresc, 2) * sizeof(uint64_t)));
    }
    // Messages go in pieces of at most kPiece bytes: a single 7.9 GB self
    // send/recv (a C3 shard's table at one rank) arrived corrupted; both sides
    // cut a slice the same way, and a group holds at most kGroupOps operations.
    constexpr uint64_t kPiece = uint64_t(1) << 30;
    struct Op {
        bool send;
        void *buf;
        uint64_t count;
        ncclDataType_t type;
        int peer;
    };
    std::vector<Op> ops;
    auto add = [&](bool send, const void *buf, uint64_t count, ncclDataType_t type, size_t esize, int peer) {
        const uint64_t per = kPiece / esize;
        for (uint64_t o = 0; o < count; o += per)
            ops.push_back(Op{send, (uint8_t *)const_cast<void *>(buf) + o * esize, std::min(per, count - o), type, peer});
    };
    for (uint32_t r = 0; r < P; ++r) {
        if (ss[r]) add(true, dk + cut[r], ss[r], ncclUint64, 8, (int)r);
        if (rs[r]) add(false, m->rk.as<uint64_t>() + roff[r], rs[r], ncclUint64, 8, (int)r);
        if (set) continue;
        if (ss[r]) add(true, m->low.as<uint8_t>() + cut[r], ss[r], ncclUint8, 1, (int)r);
        if (rs[r]) add(false, m->rlow.as<uint8_t>() + roff[r], rs[r], ncclUint8, 1, (int)r);
        if (es[r]) add(true, m->esc.as<uint64_t>() + 2 * eoff[r], 2 * es[r], ncclUint64, 8, (int)r);
        if (er[r]) add(false, m->resc.as<uint64_t>() + 2 * reoff[r], 2 * er[r], ncclUint64, 8, (int)r);
    }
    // every peer issues its pieces in the same order, so the i-th send to a
    // peer matches that peer's i-th receive from us
    constexpr size_t kGroupOps = 4096;  // one group in practice (P <= 64 peers x a few pieces)
    for (size_t g0 = 0; g0 < ops.size(); g0 += kGroupOps) {
        NCCL_TRY(rccl().GroupStart());
        for (size_t i = g0; i < std::min(ops.size(), g0 + kGroupOps); ++i) {
            const Op &o = ops[i];
            if (o.send)
                NCCL_TRY(rccl().Send(o.buf, o.count, o.type, o.peer, m->nc, s));
            else
                NCCL_TRY(rccl().Recv(o.buf, o.count, o.type, o.peer, m->nc, s));
        }
        NCCL_TRY(rccl().GroupEnd());
    }
    if (!set && nrecv) {
        const uint64_t wb = (nrecv + kPackBlock - 1) / kPackBlock;
        hipLaunchKernelGGL(k_widen_counts, dim3((uint32_t)wb), dim3(256), 0, s, m->rlow.as<uint8_t>(), nrecv,
                           m->rc.as<uint64_t>());
        if (nresc) {
            OKM_TRY(m->offs.ensure(2 * (P + 1) * sizeof(ull)));
            std::vector<ull> o(2 * (P + 1));
            std::copy(reoff.begin(), reoff.end(), o.begin());
            std::copy(roff.begin(), roff.end(), o.begin() + P + 1);
            HIP_TRY(hipMemcpyAsync(m->offs.p, o.data(), o.size() * sizeof(ull), hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_apply_escapes, dim3((uint32_t)((nresc + 255) / 256)), dim3(256), 0, s,
                               m->resc.as<uint64_t>(), nresc, m->offs.as<ull>(), m->offs.as<ull>() + P + 1, P,
                               m->rc.as<uint64_t>());
        }
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipStreamSynchronize(s));  // received: the owner's stream may read the slices
    const double t_x = ms_since(t0);

    // 5. the owner counts the P sorted slices in place (key-range items)
    OKM_TRY(okm_reset(owner));
    for (uint32_t r = 0; r < P; ++r) {
        if (r == me && self_borrow && self_n) {
            OKM_TRY(okm_add_sorted_pairs_device(owner, dk + cut[me], set ? nullptr : dc + cut[me], self_n));
            continue;
        }
        if (!rs[r]) continue;
        OKM_TRY(okm_add_sorted_pairs_device(owner, m->rk.as<uint64_t>() + roff[r],
                                            set ? nullptr : m->rc.as<uint64_t>() + roff[r], rs[r]));
    }
    uint64_t nd = 0;
    OKM_TRY(okm_count(owner, &nd));  // synchronous: the slices may be overwritten by the next call
    if (n_owned) *n_owned = nd;
    const double t_all = ms_since(t0);
    m->last_ms[0] = t_plan;
    m->last_ms[1] = t_x - t_plan;
    m->last_ms[2] = 0;
    m->last_ms[3] = t_all - t_x;
    return OKM_OK;
}

}  // extern "C"
