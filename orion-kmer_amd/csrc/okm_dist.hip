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
//   2. all-reduce of the histogram; the host cuts it into count-balanced
//      contiguous key ranges, one per rank (okm_owner_bounds: value-range
//      ownership, so the global table is the concatenation of the owners'
//      ranges in rank order and needs no final merge; canonical k-mers are
//      skewed ~7:5:3:1 by first base, so equal-width ranges would not balance);
//   3. the local table splits at the range starts (binary search again) and
//      moves with grouped point-to-point sends: keys as u64, counts as ONE
//      byte (k_pack_counts: the low byte; a count > 255 also travels as an
//      escape (position, value) that overwrites the byte on arrival,
//      k_apply_escapes): 9 B per pair on a point-to-point xGMI link instead of
//      16;
//   4. the owner adds every rank's slice — each one sorted — without copying
//      (okm_add_sorted_pairs_device) and counts them as key-range items split
//      out of every slice by binary search: counts add, the fetch_add of
//      count.rs:31-34.
//
// The collectives go through a Transport with two implementations that share
// everything above (plan, pack / widen / escape kernels, piece cutting, owner
// merge):
//   - RcclTransport: RCCL (loaded at run time with dlopen, so the library
//     still loads where no RCCL is installed; only the okm_comm_* calls then
//     fail, with OKM_E_COMM), one rank per GPU;
//   - LoopTransport: P virtual ranks in one process on one device, exchanging
//     by device copies between the ranks' buffers (host threads meet at a
//     barrier per collective).  RCCL refuses two ranks on one GPU, so this is
//     how the P > 1 code paths run on a one-GPU box (tests, rehearsals).
//
// Failure agreement: a rank that fails between collectives (e.g. out of
// memory while sizing its receive buffers) still takes part in the next
// collective with a status word set, so every rank leaves okm_merge_owned
// with an error instead of its peers blocking forever; only a failure inside
// a grouped send/recv aborts the communicator (ncclCommAbort / the loopback
// hub's abort), after which it is unusable.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "okm_dev_common.h"
#include "okm_hip_try.h"
#include "orion_kmer_testing.h"

namespace okm {

// ---------------------------------------------------------------------------
// RCCL entry points (dlopen)
// ---------------------------------------------------------------------------
struct Rccl {
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
    // what a communicator reports about itself (okm_comm_get_info; optional)
    ncclResult_t (*CommCount)(const ncclComm_t, int *) = nullptr;
    ncclResult_t (*CommUserRank)(const ncclComm_t, int *) = nullptr;
    ncclResult_t (*CommCuDevice)(const ncclComm_t, int *) = nullptr;
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
    sym(r.CommAbort, "ncclCommAbort");
    sym(r.AllReduce, "ncclAllReduce");
    sym(r.AllGather, "ncclAllGather");
    sym(r.Send, "ncclSend");
    sym(r.Recv, "ncclRecv");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.GetErrorString, "ncclGetErrorString");
    r.ok = all;
    r.CommCount = reinterpret_cast<decltype(r.CommCount)>(dlsym(h, "ncclCommCount"));
    r.CommUserRank = reinterpret_cast<decltype(r.CommUserRank)>(dlsym(h, "ncclCommUserRank"));
    r.CommCuDevice = reinterpret_cast<decltype(r.CommCuDevice)>(dlsym(h, "ncclCommCuDevice"));
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

// hist[b] += instances of bin b (several tables add into one histogram)
__global__ void k_hist_from_starts(const ull *__restrict__ starts, uint32_t nb, ull *__restrict__ hist) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) hist[b] += starts[b + 1] - starts[b];
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

// dst[i] += src[i] (the loopback all-reduce; delta decoding)
__global__ void k_add_u64(ull *__restrict__ dst, const ull *__restrict__ src, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] += src[i];
}

// Keys on the wire as 5-byte deltas.  Every destination slice of the sorted
// table is ascending, so a key travels as its difference to the slice's
// previous key (the slice's first key: to 0): the low 40 bits in 5 bytes, and
// a difference of 2^40 or more (every slice's first key, rare gaps) also as a
// key escape (position in the destination's run, difference >> 40).  The
// receiver widens the 5-byte stream, adds the escapes' high parts and
// prefix-sums each slice (okm_merge_owned step 3).  A table of ~1.4 G keys
// over the 2^61 canonical k=31 keys has gaps of ~2^31: 6 B per pair with the
// count byte instead of 9.  kDeltaPer keys per thread: 40 bytes = five
// 8-byte words (5 * 8 keys is 8-byte aligned).
constexpr int kDeltaPer = 8;
constexpr uint64_t kDeltaBlock = 256 * kDeltaPer;
constexpr uint64_t kLow40 = (uint64_t(1) << 40) - 1;

template <bool WRITE>
__global__ __launch_bounds__(256) void k_pack_deltas(const uint64_t *__restrict__ keys, uint64_t n,
                                                     const ull *__restrict__ cut, uint32_t P, uint8_t *__restrict__ out5,
                                                     ull *__restrict__ esc_cnt, ull *__restrict__ esc_cur,
                                                     uint64_t *__restrict__ esc, uint64_t skip0, uint64_t skip1) {
    const uint64_t b0 = (uint64_t)blockIdx.x * kDeltaBlock;
    if (b0 >= skip0 && b0 + kDeltaBlock <= skip1) return;  // block-uniform: the borrowed self slice
    const uint64_t i0 = b0 + (uint64_t)threadIdx.x * kDeltaPer;
    if (i0 >= n) return;
    uint32_t d = dest_of(cut, P, i0);
    uint64_t prev = i0 ? keys[i0 - 1] : 0ull;
    uint64_t w[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < kDeltaPer; ++j) {
        const uint64_t i = i0 + j;
        if (i < n) {
            while (i >= cut[d + 1]) ++d;  // empty slices are skipped; i < n = cut[P]
            const uint64_t k = keys[i];
            const uint64_t delta = k - (i == cut[d] ? 0ull : prev);
            prev = k;
            if (i < skip0 || i >= skip1) {
                if (delta >> 40) {
                    if (WRITE) {
                        const ull sidx = atomicAdd(&esc_cur[d], 1ull);
                        esc[2 * sidx] = i - cut[d];
                        esc[2 * sidx + 1] = delta >> 40;
                    } else {
                        atomicAdd(&esc_cnt[d], 1ull);
                    }
                }
                const uint64_t lo = delta & kLow40;
                const int bit = 40 * j, wi = bit >> 6, sh = bit & 63;  // compile-time
                w[wi] |= lo << sh;
                if (sh > 24) w[wi + 1] |= lo >> (64 - sh);
            }
        }
    }
    if (WRITE) return;  // the bytes are written by the counting pass
    if (i0 + kDeltaPer <= n) {
        uint64_t *o = reinterpret_cast<uint64_t *>(out5 + 5 * i0);
#pragma unroll
        for (int q = 0; q < 5; ++q) o[q] = w[q];
    } else {
        const uint64_t nb = 5 * (n - i0);
        for (uint64_t b = 0; b < nb; ++b) out5[5 * i0 + b] = (uint8_t)(w[b >> 3] >> (8 * (b & 7)));
    }
}

// 5-byte stream -> u64 deltas (the low 40 bits; escapes add the rest)
__global__ __launch_bounds__(256) void k_widen_deltas(const uint8_t *__restrict__ in5, uint64_t n,
                                                      uint64_t *__restrict__ out) {
    const uint64_t i0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * kDeltaPer;
    if (i0 >= n) return;
    uint64_t w[5] = {0, 0, 0, 0, 0};
    if (i0 + kDeltaPer <= n) {
        const uint64_t *p = reinterpret_cast<const uint64_t *>(in5 + 5 * i0);
#pragma unroll
        for (int q = 0; q < 5; ++q) w[q] = p[q];
    } else {
        const uint64_t nb = 5 * (n - i0);
        for (uint64_t b = 0; b < nb; ++b) w[b >> 3] |= (uint64_t)in5[5 * i0 + b] << (8 * (b & 7));
    }
#pragma unroll
    for (int j = 0; j < kDeltaPer; ++j) {
        const int bit = 40 * j, wi = bit >> 6, sh = bit & 63;
        uint64_t v = w[wi] >> sh;
        if (sh > 24) v |= w[wi + 1] << (64 - sh);
        if (i0 + j < n) out[i0 + j] = v & kLow40;
    }
}

// Key escapes received from rank s sit at esc[2 * reoff[s] ..]: deltas[roff[s] + pos] += high << 40.
__global__ void k_apply_key_escapes(const uint64_t *__restrict__ esc, uint64_t nesc, const ull *__restrict__ reoff,
                                    const ull *__restrict__ roff, uint32_t P, uint64_t *__restrict__ deltas) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nesc) return;
    const uint32_t s = dest_of(reoff, P, j);
    deltas[roff[s] + esc[2 * j]] += esc[2 * j + 1] << 40;
}

// ---------------------------------------------------------------------------
// Transports
// ---------------------------------------------------------------------------

// One point-to-point operation of a grouped exchange (esize: 1 = u8, 8 = u64).
struct P2POp {
    bool send;
    void *buf;
    uint64_t count;
    int esize;
    int peer;
};

class Transport {
  public:
    virtual ~Transport() = default;
    // recv[i] = sum over ranks of send[i]; send and recv are device u64 arrays
    virtual okm_status all_reduce_sum(const ull *send, ull *recv, size_t n, hipStream_t s) = 0;
    // recv[r * n + i] = rank r's send[i]
    virtual okm_status all_gather(const ull *send, ull *recv, size_t n, hipStream_t s) = 0;
    // one group of sends and receives; the i-th send from a to b matches b's
    // i-th receive from a (both sides issue their operations in one order)
    virtual okm_status exchange(const std::vector<P2POp> &ops, hipStream_t s) = 0;
    // after a failure inside a collective: peers blocked in one return an error
    virtual void abort() = 0;
    virtual const char *name() const = 0;
    // ranks, this rank and its device as the transport itself reports them
    // (RCCL: ncclCommCount / ncclCommUserRank / ncclCommCuDevice); -1 unknown
    virtual void self_report(int *count, int *rank, int *device) const = 0;
    // true: send buffers must be plain hipMalloc memory of the communicator
    // (the counting contexts' tables live in a virtual-memory arena, which
    // RCCL's peer-to-peer paths are not given to register or map)
    virtual bool owned_send_buffers() const { return false; }
};

class RcclTransport final : public Transport {
  public:
    explicit RcclTransport(ncclComm_t nc) : nc_(nc) {}
    bool owned_send_buffers() const override { return true; }
    ~RcclTransport() override {
        if (nc_) (void)rccl().CommDestroy(nc_);
    }
    okm_status all_reduce_sum(const ull *send, ull *recv, size_t n, hipStream_t s) override {
        NCCL_TRY(rccl().AllReduce(send, recv, n, ncclUint64, ncclSum, nc_, s));
        return OKM_OK;
    }
    okm_status all_gather(const ull *send, ull *recv, size_t n, hipStream_t s) override {
        NCCL_TRY(rccl().AllGather(send, recv, n, ncclUint64, nc_, s));
        return OKM_OK;
    }
    okm_status exchange(const std::vector<P2POp> &ops, hipStream_t s) override {
        NCCL_TRY(rccl().GroupStart());
        ncclResult_t bad = ncclSuccess;
        for (const P2POp &o : ops) {
            const ncclDataType_t t = o.esize == 1 ? ncclUint8 : ncclUint64;
            bad = o.send ? rccl().Send(o.buf, o.count, t, o.peer, nc_, s) : rccl().Recv(o.buf, o.count, t, o.peer, nc_, s);
            if (bad != ncclSuccess) break;
        }
        const ncclResult_t end = rccl().GroupEnd();  // the group is always closed
        if (bad != ncclSuccess) return fail(OKM_E_COMM, std::string("ncclSend/ncclRecv: ") + rccl().GetErrorString(bad));
        if (end != ncclSuccess) return fail(OKM_E_COMM, std::string("ncclGroupEnd: ") + rccl().GetErrorString(end));
        return OKM_OK;
    }
    void abort() override {
        if (nc_) (void)rccl().CommAbort(nc_);
        nc_ = nullptr;
    }
    const char *name() const override { return "rccl"; }
    void self_report(int *count, int *rank, int *device) const override {
        *count = *rank = *device = -1;
        if (!nc_) return;
        if (rccl().CommCount && rccl().CommCount(nc_, count) != ncclSuccess) *count = -1;
        if (rccl().CommUserRank && rccl().CommUserRank(nc_, rank) != ncclSuccess) *rank = -1;
        if (rccl().CommCuDevice && rccl().CommCuDevice(nc_, device) != ncclSuccess) *device = -1;
    }

  private:
    ncclComm_t nc_;
};

// The meeting point of a loopback communicator's P virtual ranks: a
// generation barrier (with a timeout, so a rank that never arrives ends the
// collective with an error instead of a hang) and the buffers each rank posts.
struct LoopHub {
    int P;
    std::mutex mu;
    std::condition_variable cv;
    uint64_t gen = 0;
    int arrived = 0;
    bool aborted = false;
    std::vector<const void *> post;           // all-reduce / all-gather sources
    std::vector<std::vector<P2POp>> sends;    // each rank's sends of the current group
    explicit LoopHub(int n) : P(n), post(n, nullptr), sends(n) {}

    static double timeout_s() {  // OKM_TEST_LOOPBACK_TIMEOUT_MS (tests), else 300 s
        const int64_t ms = test_knob(OKM_TEST_LOOPBACK_TIMEOUT_MS);
        return ms > 0 ? (double)ms * 1e-3 : 300.0;
    }
    // false: aborted (now or while waiting) or timed out (the hub is then aborted)
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) return false;
        const uint64_t g = gen;
        if (++arrived == P) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        const bool ok = cv.wait_for(lk, std::chrono::duration<double>(timeout_s()),
                                    [&] { return gen != g || aborted; });
        if (gen != g) return true;
        if (!ok) {  // timed out: nobody else is coming
            aborted = true;
            cv.notify_all();
        }
        return false;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
};

class LoopTransport final : public Transport {
  public:
    LoopTransport(std::shared_ptr<LoopHub> hub, int rank) : hub_(std::move(hub)), me_(rank) {}
    okm_status all_reduce_sum(const ull *send, ull *recv, size_t n, hipStream_t s) override {
        HIP_TRY(hipStreamSynchronize(s));
        hub_->post[me_] = send;
        if (!hub_->barrier()) return lost();
        okm_status st = OKM_OK;
        if (n) {
            (void)hipGetLastError();  // a stale (handled) error of this thread is not the launch's
            hipError_t e = hipMemcpyAsync(recv, hub_->post[0], n * sizeof(ull), hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) st = fail(OKM_E_DEVICE, std::string("loopback all-reduce: copy: ") + hipGetErrorString(e));
            for (int r = 1; r < hub_->P && st == OKM_OK; ++r) {
                hipLaunchKernelGGL(k_add_u64, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, recv,
                                   static_cast<const ull *>(hub_->post[r]), (uint64_t)n);
                e = hipGetLastError();
                if (e != hipSuccess) st = fail(OKM_E_DEVICE, std::string("loopback all-reduce: kernel: ") + hipGetErrorString(e));
            }
            if (hipStreamSynchronize(s) != hipSuccess && st == OKM_OK) st = fail(OKM_E_DEVICE, "loopback all-reduce");
        }
        return finish(st);  // sources stay unchanged until every rank has read them
    }
    okm_status all_gather(const ull *send, ull *recv, size_t n, hipStream_t s) override {
        HIP_TRY(hipStreamSynchronize(s));
        hub_->post[me_] = send;
        if (!hub_->barrier()) return lost();
        okm_status st = OKM_OK;
        for (int r = 0; r < hub_->P && st == OKM_OK && n; ++r)
            if (hipMemcpyAsync(recv + (size_t)r * n, hub_->post[r], n * sizeof(ull), hipMemcpyDeviceToDevice, s) !=
                hipSuccess)
                st = fail(OKM_E_DEVICE, "loopback all-gather: copy");
        if (hipStreamSynchronize(s) != hipSuccess && st == OKM_OK) st = fail(OKM_E_DEVICE, "loopback all-gather");
        return finish(st);
    }
    okm_status exchange(const std::vector<P2POp> &ops, hipStream_t s) override {
        HIP_TRY(hipStreamSynchronize(s));  // the sends' bytes are ready
        std::vector<P2POp> mine;
        for (const P2POp &o : ops)
            if (o.send) mine.push_back(o);
        hub_->sends[me_] = std::move(mine);
        if (!hub_->barrier()) return lost();
        // receive: the j-th receive from peer p takes p's j-th send to me
        std::vector<size_t> taken(hub_->P, 0);
        okm_status st = OKM_OK;
        for (const P2POp &o : ops) {
            if (o.send) continue;
            const std::vector<P2POp> &ps = hub_->sends[o.peer];
            size_t j = taken[o.peer], seen = 0, at = ps.size();
            for (size_t i = 0; i < ps.size(); ++i)
                if (ps[i].peer == me_ && seen++ == j) {
                    at = i;
                    break;
                }
            if (at == ps.size()) {
                st = fail(OKM_E_COMM, "loopback exchange: rank " + std::to_string(o.peer) + " posted no matching send");
                break;
            }
            const P2POp &src = ps[at];
            if (src.count != o.count || src.esize != o.esize) {
                st = fail(OKM_E_COMM, "loopback exchange: send/receive size mismatch with rank " + std::to_string(o.peer));
                break;
            }
            taken[o.peer] = j + 1;
            if (o.count && hipMemcpyAsync(o.buf, src.buf, o.count * (uint64_t)o.esize, hipMemcpyDeviceToDevice, s) !=
                               hipSuccess) {
                st = fail(OKM_E_DEVICE, "loopback exchange: copy");
                break;
            }
        }
        if (hipStreamSynchronize(s) != hipSuccess && st == OKM_OK) st = fail(OKM_E_DEVICE, "loopback exchange");
        return finish(st);  // senders may reuse their buffers once every rank has copied
    }
    void abort() override { hub_->abort(); }
    const char *name() const override { return "loopback"; }
    void self_report(int *count, int *rank, int *device) const override {
        *count = hub_->P;
        *rank = me_;
        *device = -1;  // every virtual rank shares the caller's device (okm_comm_get_info: device)
    }

  private:
    okm_status lost() { return fail(OKM_E_COMM, "loopback communicator aborted (a peer rank failed or timed out)"); }
    okm_status finish(okm_status st) {
        if (st != OKM_OK) {  // peers may wait in the closing barrier: release them
            hub_->abort();
            return st;
        }
        return hub_->barrier() ? OKM_OK : lost();
    }
    std::shared_ptr<LoopHub> hub_;
    int me_;
};

// Bytes per point-to-point message piece (512 MiB; OKM_TEST_PIECE_BYTES
// smaller in tests).  RCCL 2.27.7 (ROCm 7.2) delivers only the FIRST HALF of a
// self send/recv above 1 GiB -- every byte from size/2 on is left unwritten,
// for u8 and u64 messages alike (1.5 GiB, 2 GiB, 4 GiB, 7.9 GB all lose their
// second half; 1 GiB arrives intact: tools/rccl_big_p2p.hip,
// profiles/r03_rccl_self_p2p_sizes.txt) -- so pieces stay well below 1 GiB.
static uint64_t piece_bytes() {
    constexpr uint64_t kMax = uint64_t(1) << 29;
    const int64_t v = test_knob(OKM_TEST_PIECE_BYTES);
    return v >= 8 ? std::min<uint64_t>((uint64_t)v & ~uint64_t(7), kMax) : kMax;
}

}  // namespace okm

using namespace okm;

// ---------------------------------------------------------------------------
// Communicator
// ---------------------------------------------------------------------------
namespace {
// A communicator's device buffer (plain hipMalloc, outside the contexts'
// arenas): its bytes count against the per-device budget (OKM_HBM_CAP), so
// the contexts on the device see that much less room.  Past the budget the
// contexts' idle arena chunks are unmapped first.
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int dev = 0;
    okm_status ensure(size_t bytes) {
        if (bytes <= cap) return OKM_OK;
        release();
        const size_t want = std::max<size_t>(bytes + bytes / 8, 4096);
        (void)hipGetDevice(&dev);
        if (device_over_budget(dev, want)) trim_device_pools(dev);
        if (hipMalloc(&p, want) != hipSuccess) {
            // HBM held by the contexts' cached (idle) arena chunks: give it back, once
            (void)hipGetLastError();
            trim_device_pools(dev);
            p = nullptr;
            HIP_TRY(hipMalloc(&p, want));
        }
        cap = want;
        device_bytes_add(dev, (int64_t)cap);
        return OKM_OK;
    }
    template <typename T> T *as() const { return static_cast<T *>(p); }
    void release() {
        if (p) {
            (void)hipFree(p);
            device_bytes_add(dev, -(int64_t)cap);
        }
        p = nullptr;
        cap = 0;
    }
};
}  // namespace

struct okm_comm {
    int device = 0, rank = 0, size = 1;
    std::unique_ptr<Transport> tp;
    bool broken = false;  // aborted after a failure inside a collective
    hipStream_t stream = nullptr;
    DevBuf starts, hist, hsum, cut, sizes, gsizes, low, esc_cnt, esc_cur, esc, rk, rlow, rc, resc, offs, flag;
    DevBuf k5, kesc, kesc_cur, rk5, rkesc, stmp;  // keys as 5-byte deltas (+ key escapes, scan scratch)
    DevBuf ksend;  // u64 keys sent from communicator memory (Transport::owned_send_buffers)
    ull *hpin = nullptr;  // pinned landing area for the small readbacks
    size_t hpin_cap = 0;
    // the agreed histogram over this rank's owner range (zero elsewhere): the
    // owner's count plans its items from it (set_sorted_hint)
    std::vector<ull> owned_hist;
    double last_ms[4] = {0, 0, 0, 0};  // plan, exchange, unpack, merge (host wall, last okm_merge_owned)
    uint64_t last_bytes[2] = {0, 0};   // bytes sent / received by the last okm_merge_owned (excl. self)
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

// A failure inside a collective leaves peers in undefined places: the
// communicator is aborted and refuses further merges.
okm_status broke(okm_comm *m, okm_status st) {
    m->tp->abort();
    m->broken = true;
    return st;
}

// Test hook: OKM_TEST_FAIL_RANK = r makes rank r fail while sizing its receive
// buffers (after the size exchange, before any send): every rank must return
// an error and the communicator must stay usable.
int debug_fail_rank() { return (int)test_knob(OKM_TEST_FAIL_RANK); }

// One local table taking part in a merge.
struct Table {
    okm_ctx *local, *owner;
    const uint64_t *dk = nullptr, *dc = nullptr;
    uint64_t n = 0;
    std::vector<ull> starts;  // first index of every top-bits bin (nb + 1)
};

// Steps 1-2 (see the file comment) for nt tables at once: their histograms
// summed, then over ranks; the owner split balances the sum, so equal keys of
// different tables meet on one rank.  Returns with every rank agreeing on
// success: the word nb of the all-reduce carries "this rank failed".
// Keys as 5-byte deltas on the wire: OKM_TEST_WIRE_DELTAS = 1 / 0 forces either;
// by default (2) with 2 to 4 ranks, where one to three xGMI links per GPU
// bound the exchange and 9 -> 6 B per pair pays for the receiver's decode
// passes (with 8 ranks and seven links per GPU the decode costs about what
// the bytes save), and only for tables dense enough that gaps of 2^40 and
// more (16-B key escapes) are rare: a rank's table (the agreed histogram's
// total / P) leaves a mean gap of at most 2^38 over the 2^(2k-1) canonical
// keys (an exponential gap passes 2^40 with probability e^-4: +0.3 B a pair).
int want_deltas(uint32_t P) {
    const int64_t e = test_knob(OKM_TEST_WIRE_DELTAS);
    if (e >= 0) return e != 0 ? 1 : 0;
    return P > 1 && P <= 4 ? 2 : 0;
}
bool dense_enough(uint64_t pairs_per_rank, uint32_t k) {
    const uint32_t space_bits = 2 * k - 1;  // canonical keys: about half of the 2k-bit values
    return space_bits <= 38 || (double)pairs_per_rank >= std::ldexp(1.0, (int)space_bits - 38);
}

okm_status plan_split(okm_comm *m, std::vector<Table> &tabs, uint32_t nb, uint32_t shift, std::vector<uint32_t> &bounds,
                      bool *deltas) {
    const uint32_t P = (uint32_t)m->size;
    const size_t nt = tabs.size();
    hipStream_t s = m->stream;
    // The small buffers every collective needs: without them this rank cannot
    // even report its failure to its peers, so the communicator is aborted.
    {
        okm_status a = OKM_OK;
        for (auto [b, bytes] : {std::pair<DevBuf *, size_t>{&m->starts, nt * (nb + 1) * sizeof(ull)},
                                {&m->hist, (nb + 3) * sizeof(ull)},
                                {&m->hsum, (nb + 3) * sizeof(ull)},
                                {&m->cut, (P + 1) * sizeof(ull)},
                                {&m->sizes, (3 * P + 1) * sizeof(ull)},
                                {&m->gsizes, (3 * (size_t)P + 1) * P * sizeof(ull)},
                                {&m->esc_cnt, P * sizeof(ull)},
                                {&m->esc_cur, (P + 1) * sizeof(ull)},
                                {&m->kesc_cur, (P + 1) * sizeof(ull)},
                                {&m->offs, 4 * (P + 1) * sizeof(ull)},
                                {&m->flag, 2 * sizeof(ull)}})
            if (a == OKM_OK) a = b->ensure(bytes);
        if (a == OKM_OK) a = ensure_hpin(m, (nt + 1) * (nb + 3) + (3 * (size_t)P + 1) * P + 64);
        if (a != OKM_OK) return broke(m, a);
    }
    // host sources of async copies: live until the sync below
    const ull one = 1;
    const bool wide = ctx_is_wide(tabs[0].local);  // K128 keys (k > 32): u64 word pairs, never deltas
    // words nb + 1 / nb + 2 of the all-reduce: ranks that want deltas (forced
    // or auto) / ranks that FORCE them.  Both must be 0 or P: a forced rank
    // beside an auto rank would otherwise pick a different format than its peer
    const int wmode = wide ? 0 : want_deltas(P);
    const ull wd[2] = {wmode ? 1ull : 0ull, wmode == 1 ? 1ull : 0ull};
    okm_status st = OKM_OK;
    for (size_t i = 0; i < nt && st == OKM_OK; ++i)  // counts the local shards if needed (synchronous)
        st = okm_result_device(tabs[i].local, &tabs[i].dk, &tabs[i].dc, &tabs[i].n);
    HIP_TRY(hipMemsetAsync(m->hist.p, 0, (nb + 1) * sizeof(ull), s));
    HIP_TRY(hipMemcpyAsync(m->hist.as<ull>() + nb + 1, wd, 2 * sizeof(ull), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(m->starts.p, 0, nt * (nb + 1) * sizeof(ull), s));
    if (st == OKM_OK) {
        for (size_t i = 0; i < nt; ++i) {
            ull *st_i = m->starts.as<ull>() + i * (nb + 1);
            launch_bin_bounds(s, tabs[i].dk, tabs[i].n, shift, nb, st_i, wide);
            hipLaunchKernelGGL(k_hist_from_starts, dim3((nb + 255) / 256), dim3(256), 0, s, st_i, nb,
                               m->hist.as<ull>());
            HIP_TRY(hipGetLastError());
        }
    } else {
        HIP_TRY(hipMemcpyAsync(m->hist.as<ull>() + nb, &one, sizeof(ull), hipMemcpyHostToDevice, s));
    }
    {
        okm_status c = m->tp->all_reduce_sum(m->hist.as<ull>(), m->hsum.as<ull>(), nb + 3, s);
        if (c != OKM_OK) return broke(m, c);
    }
    ull *h_sum = m->hpin, *h_starts = m->hpin + nb + 3;
    HIP_TRY(hipMemcpyAsync(h_sum, m->hsum.p, (nb + 3) * sizeof(ull), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(h_starts, m->starts.p, nt * (nb + 1) * sizeof(ull), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (st != OKM_OK) return st;
    if (h_sum[nb]) return fail(OKM_E_COMM, "okm_merge_owned: a peer rank failed before the exchange");
    if ((h_sum[nb + 1] != 0 && h_sum[nb + 1] != P) || (h_sum[nb + 2] != 0 && h_sum[nb + 2] != P))
        return fail(OKM_E_COMM, "okm_merge_owned: ranks disagree on the key wire format (OKM_TEST_WIRE_DELTAS)");
    uint64_t pairs = 0;
    for (uint32_t b = 0; b < nb; ++b) pairs += h_sum[b];
    // every rank sees the same sums: the same decision everywhere
    *deltas = h_sum[nb + 1] == P && (h_sum[nb + 2] == P || dense_enough(pairs / P, ctx_k(tabs[0].local)));
    for (size_t i = 0; i < nt; ++i) tabs[i].starts.assign(h_starts + i * (nb + 1), h_starts + (i + 1) * (nb + 1));
    bounds.assign(P + 1, 0);  // (h_starts stays valid: tabs[i].starts copied above)
    owner_bounds(reinterpret_cast<const uint64_t *>(h_sum), nb, (int)P, bounds.data());
    // what this rank will own, bin by bin (h_sum is the sum over ranks of
    // every table's pairs, so for several tables an upper bound of each)
    m->owned_hist.assign(nb, 0);
    const uint32_t me = (uint32_t)m->rank;
    std::copy(h_sum + bounds[me], h_sum + bounds[me + 1], m->owned_hist.begin() + bounds[me]);
    return OKM_OK;
}

// Steps 3-4 for one table under agreed bounds: sizes, escapes, the grouped
// exchange, then the owner's count of the received slices.
okm_status move_and_merge(okm_comm *m, Table &t, const std::vector<uint32_t> &bounds, uint32_t nb, bool deltas,
                          uint64_t *n_owned, double *ms3, uint64_t *bytes2) {
    const auto t0 = std::chrono::steady_clock::now();
    okm_ctx *local = t.local, *owner = t.owner;
    const bool set = ctx_is_set(local) || ctx_is_set(owner);
    const uint32_t P = (uint32_t)m->size, me = (uint32_t)m->rank;
    hipStream_t s = m->stream;
    Transport &tp = *m->tp;
    const uint64_t *dk = t.dk, *dc = t.dc;
    const uint64_t n = t.n;
    const uint64_t kw = ctx_is_wide(local) ? 2 : 1;  // u64 words per key (K128 keys travel as word pairs)
    // host sources of async copies live until the stream is synchronised
    ull bad = 0;
    std::vector<ull> esc_offs(4 * (P + 1));
    std::vector<ull> cut(P + 1);
    for (uint32_t r = 0; r <= P; ++r) cut[r] = bounds[r] >= nb ? n : t.starts[bounds[r]];
    cut[0] = 0;
    cut[P] = n;

    // 3. sizes, count escapes and key escapes of every pair of ranks; word 3P = status
    HIP_TRY(hipMemcpyAsync(m->cut.p, cut.data(), (P + 1) * sizeof(ull), hipMemcpyHostToDevice, s));
    const size_t row = 3 * (size_t)P + 1;
    std::vector<ull> hs(row, 0);
    for (uint32_t r = 0; r < P; ++r) hs[r] = cut[r + 1] - cut[r];
    // This rank's own slice never crosses the transport when the owner is
    // another context: the owner borrows it straight from the local table (it
    // stays unchanged until okm_count(owner) returns below).  owner == local
    // receives it through a self send/recv, since okm_reset(owner) releases it.
    const bool self_borrow = owner != local;
    const uint64_t skip0 = self_borrow ? cut[me] : 0, skip1 = self_borrow ? cut[me + 1] : 0;
    const uint64_t pblocks = (n + kPackBlock - 1) / kPackBlock;
    const uint64_t dblocks = (n + kDeltaBlock - 1) / kDeltaBlock;
    okm_status st = OKM_OK;
    if (!set) st = m->low.ensure(std::max<uint64_t>(n, 16));
    if (deltas && st == OKM_OK) st = m->k5.ensure(5 * std::max<uint64_t>(n, 16));
    // u64 keys go out of communicator memory (owned_send_buffers): the slices
    // that cross the transport (not the borrowed self slice) are staged below,
    // allocated here so that a failure is still reported to the peers
    const uint64_t n_sent = n - (self_borrow ? skip1 - skip0 : 0);
    if (!deltas && st == OKM_OK && tp.owned_send_buffers())
        st = m->ksend.ensure(kw * std::max<uint64_t>(n_sent, 16) * sizeof(uint64_t));
    hs[3 * P] = st != OKM_OK;
    HIP_TRY(hipMemcpyAsync(m->sizes.p, hs.data(), row * sizeof(ull), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(m->sizes.as<ull>() + P, 0, 2 * P * sizeof(ull), s));
    if (!set && st == OKM_OK && pblocks && n_sent) {  // (n_sent == 0: nothing leaves this rank)
        hipLaunchKernelGGL(k_pack_counts<false>, dim3((uint32_t)pblocks), dim3(256), 0, s, dc, n, m->cut.as<ull>(), P,
                           m->low.as<uint8_t>(), m->sizes.as<ull>() + P, nullptr, nullptr, skip0, skip1);
        HIP_TRY(hipGetLastError());
    }
    if (deltas && st == OKM_OK && dblocks && n_sent) {
        hipLaunchKernelGGL(k_pack_deltas<false>, dim3((uint32_t)dblocks), dim3(256), 0, s, dk, n, m->cut.as<ull>(), P,
                           m->k5.as<uint8_t>(), m->sizes.as<ull>() + 2 * P, nullptr, nullptr, skip0, skip1);
        HIP_TRY(hipGetLastError());
    }
    {
        okm_status c = tp.all_gather(m->sizes.as<ull>(), m->gsizes.as<ull>(), row, s);
        if (c != OKM_OK) return broke(m, c);
    }
    std::vector<ull> h_g(row * P);
    HIP_TRY(hipMemcpyAsync(m->hpin, m->gsizes.p, row * P * sizeof(ull), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::copy(m->hpin, m->hpin + row * P, h_g.begin());
    if (st != OKM_OK) return st;
    for (uint32_t r = 0; r < P; ++r)
        if (h_g[(size_t)r * row + 3 * P]) return fail(OKM_E_COMM, "okm_merge_owned: a peer rank failed while sizing");
    // per peer: pairs sent / received, count escapes sent / received, key
    // escapes sent / received (and their offsets)
    std::vector<ull> ss(P), rs(P), es(P), er(P), ks(P), kr(P), roff(P + 1, 0), reoff(P + 1, 0), eoff(P + 1, 0),
        kroff(P + 1, 0), ksoff(P + 1, 0);
    for (uint32_t r = 0; r < P; ++r) {
        ss[r] = h_g[(size_t)me * row + r];
        es[r] = h_g[(size_t)me * row + P + r];
        ks[r] = h_g[(size_t)me * row + 2 * P + r];
        rs[r] = h_g[(size_t)r * row + me];
        er[r] = h_g[(size_t)r * row + P + me];
        kr[r] = h_g[(size_t)r * row + 2 * P + me];
        roff[r + 1] = roff[r] + rs[r];
        reoff[r + 1] = reoff[r] + er[r];
        eoff[r + 1] = eoff[r] + es[r];
        kroff[r + 1] = kroff[r] + kr[r];
        ksoff[r + 1] = ksoff[r] + ks[r];
    }
    const uint64_t self_n = ss[me];
    if (self_borrow) {
        for (uint32_t r = me + 1; r <= P; ++r) roff[r] -= rs[me], reoff[r] -= er[me], kroff[r] -= kr[me];
        rs[me] = er[me] = kr[me] = 0;
        ss[me] = es[me] = ks[me] = 0;
    }
    const uint64_t nrecv = roff[P], nresc = reoff[P], nesc = eoff[P], nkr = kroff[P], nks = ksoff[P];

    // receive buffers and the escapes, then one more status word: a rank that
    // cannot allocate them tells its peers before any send is posted
    st = m->rk.ensure(std::max<uint64_t>(nrecv, 1) * kw * sizeof(uint64_t));
    if (!set) {
        if (st == OKM_OK) st = m->rlow.ensure(std::max<uint64_t>(nrecv, 16));
        if (st == OKM_OK) st = m->resc.ensure(std::max<uint64_t>(2 * nresc, 2) * sizeof(uint64_t));
        if (st == OKM_OK && nesc) st = m->esc.ensure(2 * nesc * sizeof(uint64_t));
    }
    // rc: the received counts, and first the deltas' scan (keys decoded before the counts)
    if (st == OKM_OK && (!set || deltas)) st = m->rc.ensure(std::max<uint64_t>(nrecv, 1) * sizeof(uint64_t));
    uint64_t max_rs = 0;
    for (uint32_t r = 0; r < P; ++r) max_rs = std::max<uint64_t>(max_rs, rs[r]);
    if (deltas) {
        if (st == OKM_OK) st = m->rk5.ensure(5 * std::max<uint64_t>(nrecv, 16));
        if (st == OKM_OK) st = m->rkesc.ensure(std::max<uint64_t>(2 * nkr, 2) * sizeof(uint64_t));
        if (st == OKM_OK && nks) st = m->kesc.ensure(2 * nks * sizeof(uint64_t));
        if (st == OKM_OK) st = m->stmp.ensure(scan_tmp_elems(max_rs + 1) * sizeof(ull));
    }
    if (st == OKM_OK && debug_fail_rank() == (int)me) st = fail(OKM_E_NOMEM, "okm_merge_owned: OKM_TEST_FAIL_RANK test hook");
    if (st == OKM_OK && !set && nesc) {  // escapes grouped by destination
        HIP_TRY(hipMemcpyAsync(m->esc_cur.p, eoff.data(), P * sizeof(ull), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_pack_counts<true>, dim3((uint32_t)pblocks), dim3(256), 0, s, dc, n, m->cut.as<ull>(), P,
                           m->low.as<uint8_t>(), nullptr, m->esc_cur.as<ull>(), m->esc.as<uint64_t>(), skip0, skip1);
        HIP_TRY(hipGetLastError());
    }
    if (st == OKM_OK && deltas && nks) {  // key escapes grouped by destination
        HIP_TRY(hipMemcpyAsync(m->kesc_cur.p, ksoff.data(), P * sizeof(ull), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_pack_deltas<true>, dim3((uint32_t)dblocks), dim3(256), 0, s, dk, n, m->cut.as<ull>(), P,
                           m->k5.as<uint8_t>(), nullptr, m->kesc_cur.as<ull>(), m->kesc.as<uint64_t>(), skip0, skip1);
        HIP_TRY(hipGetLastError());
    }
    if (P > 1) {
        bad = st != OKM_OK;
        HIP_TRY(hipMemcpyAsync(m->flag.p, &bad, sizeof(ull), hipMemcpyHostToDevice, s));
        okm_status c = tp.all_reduce_sum(m->flag.as<ull>(), m->flag.as<ull>() + 1, 1, s);
        if (c != OKM_OK) return broke(m, c);
        HIP_TRY(hipMemcpyAsync(m->hpin, m->flag.as<ull>() + 1, sizeof(ull), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (st != OKM_OK) return st;
        if (m->hpin[0]) return fail(OKM_E_COMM, "okm_merge_owned: a peer rank failed to allocate its receive buffers");
    } else if (st != OKM_OK) {
        return st;
    }
    const double t_plan = ms_since(t0);

    // 4. move the slices: keys as u64, counts as bytes (+ escapes), in pieces
    // of at most piece_bytes().  Group j holds piece j of every message, so a
    // group's sends and receives always match their peers' group j (a group
    // cut by operation count could pair a send of one group with a receive of
    // a later one on the peer and deadlock).
    struct Msg {
        bool send;
        uint8_t *buf;
        uint64_t count;
        int esize;
        int peer;
    };
    std::vector<Msg> msgs;
    auto add = [&](bool send, const void *buf, uint64_t count, int esize, uint32_t peer) {
        if (count) msgs.push_back(Msg{send, (uint8_t *)const_cast<void *>(buf), count, esize, (int)peer});
    };
    uint64_t bytes_out = 0, bytes_in = 0;
    // u64 keys: the local table's slices in place, or (owned_send_buffers) each
    // sent slice staged at sst[r] of the communicator's buffer -- only what
    // crosses the transport: nothing at one rank, (P-1)/P of the table at P
    std::vector<uint64_t> sst(P, 0);
    const uint64_t *ksrc = dk;
    const bool staged = !deltas && tp.owned_send_buffers();
    if (staged) {
        uint64_t at = 0;
        for (uint32_t r = 0; r < P; ++r) {
            sst[r] = at;
            if (ss[r])
                HIP_TRY(hipMemcpyAsync(m->ksend.as<uint64_t>() + kw * at, dk + kw * cut[r], kw * ss[r] * sizeof(uint64_t),
                                       hipMemcpyDeviceToDevice, s));
            at += ss[r];
        }
        ksrc = m->ksend.as<uint64_t>();
    } else {
        for (uint32_t r = 0; r < P; ++r) sst[r] = cut[r];
    }
    for (uint32_t r = 0; r < P; ++r) {
        if (deltas) {  // 5 bytes per key + key escapes
            add(true, m->k5.as<uint8_t>() + 5 * cut[r], 5 * ss[r], 1, r);
            add(false, m->rk5.as<uint8_t>() + 5 * roff[r], 5 * rs[r], 1, r);
            add(true, m->kesc.as<uint64_t>() + 2 * ksoff[r], 2 * ks[r], 8, r);
            add(false, m->rkesc.as<uint64_t>() + 2 * kroff[r], 2 * kr[r], 8, r);
        } else {
            add(true, ksrc + kw * sst[r], kw * ss[r], 8, r);
            add(false, m->rk.as<uint64_t>() + kw * roff[r], kw * rs[r], 8, r);
        }
        if (!set) {
            add(true, m->low.as<uint8_t>() + cut[r], ss[r], 1, r);
            add(false, m->rlow.as<uint8_t>() + roff[r], rs[r], 1, r);
            add(true, m->esc.as<uint64_t>() + 2 * eoff[r], 2 * es[r], 8, r);
            add(false, m->resc.as<uint64_t>() + 2 * reoff[r], 2 * er[r], 8, r);
        }
        if (r != me) {
            const uint64_t kb = deltas ? 5 : 8 * kw;
            bytes_out += ss[r] * (kb + (set ? 0 : 1)) + (set ? 0 : 16 * es[r]) + (deltas ? 16 * ks[r] : 0);
            bytes_in += rs[r] * (kb + (set ? 0 : 1)) + (set ? 0 : 16 * er[r]) + (deltas ? 16 * kr[r] : 0);
        }
    }
    // every rank runs the same number of groups: the most pieces of ANY
    // message between any two ranks (the all-gathered sizes), so the loopback
    // barriers pair up; an RCCL group with nothing of this rank's in it is empty
    const uint64_t piece = piece_bytes();
    uint64_t npieces = 0;
    for (uint32_t a = 0; a < P; ++a)
        for (uint32_t b = 0; b < P; ++b) {  // a == b too: whether a rank's owner borrows is its own choice
            const uint64_t pairs = h_g[(size_t)a * row + b], ce = h_g[(size_t)a * row + P + b],
                           ke = h_g[(size_t)a * row + 2 * P + b];
            uint64_t big = pairs * (deltas ? 5 : 8 * kw);
            if (!set) big = std::max(big, std::max<uint64_t>(pairs, 16 * ce));
            if (deltas) big = std::max<uint64_t>(big, 16 * ke);
            npieces = std::max<uint64_t>(npieces, (big + piece - 1) / piece);
        }
    std::vector<P2POp> ops;
    for (uint64_t j = 0; j < npieces; ++j) {
        ops.clear();
        for (const Msg &g : msgs) {
            const uint64_t per = piece / (uint64_t)g.esize, o = j * per;
            if (o < g.count) ops.push_back(P2POp{g.send, g.buf + o * g.esize, std::min(per, g.count - o), g.esize, g.peer});
        }
        okm_status c = tp.exchange(ops, s);
        if (c != OKM_OK) return broke(m, c);
    }
    if (deltas && nrecv) {
        // keys: 40-bit deltas widened, escapes' high parts added, then every
        // source rank's slice prefix-summed (exclusive scan into rc, rk += rc)
        const uint64_t db = (nrecv + kDeltaBlock - 1) / kDeltaBlock;
        hipLaunchKernelGGL(k_widen_deltas, dim3((uint32_t)db), dim3(256), 0, s, m->rk5.as<uint8_t>(), nrecv,
                           m->rk.as<uint64_t>());
        if (nkr) {
            std::copy(kroff.begin(), kroff.end(), esc_offs.begin() + 2 * (P + 1));
            std::copy(roff.begin(), roff.end(), esc_offs.begin() + 3 * (P + 1));
            HIP_TRY(hipMemcpyAsync(m->offs.as<ull>() + 2 * (P + 1), esc_offs.data() + 2 * (P + 1),
                                   2 * (P + 1) * sizeof(ull), hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_apply_key_escapes, dim3((uint32_t)((nkr + 255) / 256)), dim3(256), 0, s,
                               m->rkesc.as<uint64_t>(), nkr, m->offs.as<ull>() + 2 * (P + 1),
                               m->offs.as<ull>() + 3 * (P + 1), P, m->rk.as<uint64_t>());
        }
        for (uint32_t r = 0; r < P; ++r)
            if (rs[r])
                launch_exclusive_scan(s, m->rk.as<ull>() + roff[r], m->rc.as<ull>() + roff[r], rs[r], m->stmp.as<ull>());
        hipLaunchKernelGGL(k_add_u64, dim3((uint32_t)((nrecv + 255) / 256)), dim3(256), 0, s, m->rk.as<ull>(),
                           m->rc.as<ull>(), nrecv);
        HIP_TRY(hipGetLastError());
    }
    if (!set && nrecv) {
        const uint64_t wb = (nrecv + kPackBlock - 1) / kPackBlock;
        hipLaunchKernelGGL(k_widen_counts, dim3((uint32_t)wb), dim3(256), 0, s, m->rlow.as<uint8_t>(), nrecv,
                           m->rc.as<uint64_t>());
        if (nresc) {
            std::copy(reoff.begin(), reoff.end(), esc_offs.begin());
            std::copy(roff.begin(), roff.end(), esc_offs.begin() + P + 1);
            HIP_TRY(hipMemcpyAsync(m->offs.p, esc_offs.data(), esc_offs.size() * sizeof(ull), hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_apply_escapes, dim3((uint32_t)((nresc + 255) / 256)), dim3(256), 0, s,
                               m->resc.as<uint64_t>(), nresc, m->offs.as<ull>(), m->offs.as<ull>() + P + 1, P,
                               m->rc.as<uint64_t>());
        }
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipStreamSynchronize(s));  // received: the owner's stream may read the slices
    const double t_x = ms_since(t0);

    // 5. the owner counts the P sorted slices in place (key-range items); no
    // collective from here on.  The agreed histogram tells the owner's plan
    // how dense each part of its range is, so its first split fits.
    OKM_TRY(okm_reset(owner));
    if (m->owned_hist.size() == nb) set_sorted_hint(owner, m->owned_hist.data(), 31 - __builtin_clz(nb));
    for (uint32_t r = 0; r < P; ++r) {
        if (r == me && self_borrow && self_n) {
            OKM_TRY(okm_add_sorted_pairs_device(owner, dk + kw * cut[me], set ? nullptr : dc + cut[me], self_n));
            continue;
        }
        if (!rs[r]) continue;
        OKM_TRY(okm_add_sorted_pairs_device(owner, m->rk.as<uint64_t>() + kw * roff[r],
                                            set ? nullptr : m->rc.as<uint64_t>() + roff[r], rs[r]));
    }
    uint64_t nd = 0;
    // synchronous; the owner releases the borrowed slices once counted, so the
    // next add / merge may overwrite them (okm_engine.hip do_count)
    OKM_TRY(okm_count(owner, &nd));
    if (n_owned) *n_owned = nd;
    ms3[0] += t_plan;
    ms3[1] += t_x - t_plan;
    ms3[2] += ms_since(t0) - t_x;
    bytes2[0] += bytes_out;
    bytes2[1] += bytes_in;
    return OKM_OK;
}

// The collective body of okm_merge_owned / okm_merge_owned_n.
okm_status merge_owned_n(okm_ctx *const *locals, okm_comm *m, okm_ctx *const *owners, int nt, uint64_t *n_owned) {
    const auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipSetDevice(m->device));
    if (m->size == 1) {
        // one rank: the owner's range is the whole key space and its only
        // slice the local table -- handed over, no exchange and no copy
        // (adopt_result; owner == local, or a local still holding runs, takes
        // the general path below)
        bool all = true;
        for (int i = 0; i < nt && all; ++i) {
            bool adopted = false;
            OKM_TRY(adopt_result(owners[i], locals[i], &adopted));
            if (adopted && n_owned) OKM_TRY(okm_count(owners[i], n_owned + i));  // (counted: returns its size)
            all = adopted;
        }
        if (all) {
            m->last_ms[0] = m->last_ms[1] = m->last_ms[2] = 0;
            m->last_ms[3] = ms_since(t0);
            m->last_bytes[0] = m->last_bytes[1] = 0;
            return OKM_OK;
        }
    }
    const uint32_t k = ctx_k(locals[0]);
    const uint32_t bits = std::min<uint32_t>(16, 2 * k);
    const uint32_t nb = 1u << bits, shift = 2 * k - bits;
    std::vector<Table> tabs(nt);
    for (int i = 0; i < nt; ++i) {
        tabs[i].local = locals[i];
        tabs[i].owner = owners[i];
    }
    std::vector<uint32_t> bounds;
    bool deltas = false;
    OKM_TRY(plan_split(m, tabs, nb, shift, bounds, &deltas));
    double ms3[3] = {ms_since(t0), 0, 0};
    uint64_t bytes2[2] = {0, 0};
    for (int i = 0; i < nt; ++i)
        OKM_TRY(move_and_merge(m, tabs[i], bounds, nb, deltas, n_owned ? n_owned + i : nullptr, ms3, bytes2));
    m->last_ms[0] = ms3[0];
    m->last_ms[1] = ms3[1];
    m->last_ms[2] = 0;
    m->last_ms[3] = ms3[2];
    m->last_bytes[0] = bytes2[0];
    m->last_bytes[1] = bytes2[1];
    return OKM_OK;
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
    ncclComm_t nc = nullptr;
    NCCL_TRY(rccl().CommInitRank(&nc, nranks, u, rank));
    okm_comm *m = new okm_comm();
    m->device = device;
    m->rank = rank;
    m->size = nranks;
    m->tp.reset(new RcclTransport(nc));
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
        m->tp.reset(new RcclTransport(ncs[i]));
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

okm_status okm_comm_init_loopback(okm_comm **out, int n, int device) {
    if (!out || n < 1) return fail(OKM_E_ARG, "okm_comm_init_loopback: bad arguments");
    auto hub = std::make_shared<LoopHub>(n);
    for (int i = 0; i < n; ++i) out[i] = nullptr;
    for (int i = 0; i < n; ++i) {
        okm_comm *m = new okm_comm();
        m->device = device;
        m->rank = i;
        m->size = n;
        m->tp.reset(new LoopTransport(hub, i));
        out[i] = m;
        okm_status st = comm_finish_init(m);
        if (st != OKM_OK) {
            for (int j = 0; j <= i; ++j) okm_comm_destroy(out[j]);
            for (int j = 0; j < n; ++j) out[j] = nullptr;
            return st;
        }
    }
    return OKM_OK;
}

void okm_comm_destroy(okm_comm *m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    m->tp.reset();
    for (DevBuf *b : {&m->starts, &m->hist, &m->hsum, &m->cut, &m->sizes, &m->gsizes, &m->low, &m->esc_cnt,
                      &m->esc_cur, &m->esc, &m->rk, &m->rlow, &m->rc, &m->resc, &m->offs, &m->flag, &m->k5, &m->kesc,
                      &m->kesc_cur, &m->rk5, &m->rkesc, &m->stmp, &m->ksend})
        b->release();
    if (m->hpin) (void)hipHostFree(m->hpin);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

int okm_comm_rank(const okm_comm *m) { return m ? m->rank : -1; }

okm_status okm_comm_get_info(const okm_comm *m, okm_comm_info *info) {
    if (!m || !info) return fail(OKM_E_ARG, "null argument");
    *info = okm_comm_info{};
    info->size = m->size;
    info->rank = m->rank;
    info->device = m->device;
    m->tp->self_report(&info->transport_ranks, &info->transport_rank, &info->transport_device);
    snprintf(info->transport, sizeof(info->transport), "%s", m->tp->name());
    if (hipDeviceGetPCIBusId(info->pci_bus_id, (int)sizeof(info->pci_bus_id), m->device) != hipSuccess) {
        (void)hipGetLastError();
        info->pci_bus_id[0] = 0;
    }
    return OKM_OK;
}
int okm_comm_size(const okm_comm *m) { return m ? m->size : 0; }

okm_status okm_comm_last_times(const okm_comm *m, double *ms4) {
    if (!m || !ms4) return fail(OKM_E_ARG, "null argument");
    for (int i = 0; i < 4; ++i) ms4[i] = m->last_ms[i];
    return OKM_OK;
}

okm_status okm_comm_last_bytes(const okm_comm *m, uint64_t *sent, uint64_t *received) {
    if (!m) return fail(OKM_E_ARG, "null argument");
    if (sent) *sent = m->last_bytes[0];
    if (received) *received = m->last_bytes[1];
    return OKM_OK;
}

okm_status okm_merge_owned_n(okm_ctx *const *locals, okm_comm *m, okm_ctx *const *owners, int n,
                             uint64_t *n_owned) {
    // argument errors are the caller's and symmetric (every rank passes the
    // same kind of contexts): they return before any collective
    if (!locals || !m || !owners || n < 1) return fail(OKM_E_ARG, "okm_merge_owned: null argument");
    if (m->broken) return fail(OKM_E_COMM, "okm_merge_owned: communicator aborted by an earlier failure");
    for (int i = 0; i < n; ++i) {
        okm_ctx *local = locals[i], *owner = owners[i];
        if (!local || !owner) return fail(OKM_E_ARG, "okm_merge_owned: null context");
        if (ctx_device(local) != m->device || ctx_device(owner) != m->device)
            return fail(OKM_E_ARG, "okm_merge_owned: local, owner and communicator must share one device");
        // owner == local is allowed (and cheapest: one context, one device
        // pool): the local table is only read until the exchange has completed
        // k > 32: K128 keys (two u64 words a key) on the wire, never 5-byte deltas
        if (ctx_k(local) != ctx_k(owner) || ctx_k(local) != ctx_k(locals[0]) ||
            ctx_is_wide(local) != ctx_is_wide(owner) || ctx_is_wide(local) != ctx_is_wide(locals[0]))
            return fail(OKM_E_ARG, "okm_merge_owned: every table must have the same k (and key width)");
        for (int j = 0; j < i; ++j)
            if (owners[j] == owner || owners[j] == local || locals[j] == owner)
                return fail(OKM_E_ARG, "okm_merge_owned_n: every table needs its own contexts");
    }
    return merge_owned_n(locals, m, owners, n, n_owned);
}

okm_status okm_merge_owned(okm_ctx *local, okm_comm *m, okm_ctx *owner, uint64_t *n_owned) {
    return okm_merge_owned_n(&local, m, &owner, 1, n_owned);
}

okm_status okm_comm_allreduce_u64(okm_comm *m, const uint64_t *in, uint64_t *out, uint32_t n) {
    if (!m || (n && (!in || !out))) return fail(OKM_E_ARG, "okm_comm_allreduce_u64: null argument");
    if (m->broken) return fail(OKM_E_COMM, "okm_comm_allreduce_u64: communicator aborted by an earlier failure");
    if (!n) return OKM_OK;
    HIP_TRY(hipSetDevice(m->device));
    okm_status st = m->flag.ensure(2 * (size_t)n * sizeof(ull));
    if (st == OKM_OK) st = ensure_hpin(m, 2 * (size_t)n);
    if (st != OKM_OK) return broke(m, st);
    hipStream_t s = m->stream;
    memcpy(m->hpin, in, n * sizeof(ull));
    HIP_TRY(hipMemcpyAsync(m->flag.p, m->hpin, n * sizeof(ull), hipMemcpyHostToDevice, s));
    st = m->tp->all_reduce_sum(m->flag.as<ull>(), m->flag.as<ull>() + n, n, s);
    if (st != OKM_OK) return broke(m, st);
    HIP_TRY(hipMemcpyAsync(m->hpin + n, m->flag.as<ull>() + n, n * sizeof(ull), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    memcpy(out, m->hpin + n, n * sizeof(ull));
    return OKM_OK;
}

}  // extern "C"
