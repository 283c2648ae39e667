// okm_group.cpp — one counting context per GPU in one process: the
// `orion-kmer count --gpus N` engine, and the host feed's pipeline.
//
// The reference's count is one thread filling one DashMap record by record
// (count.rs:48-79).  Here the CLI's reader parses the next batch while the
// GPUs count the previous ones: okm_group_add_batch copies the batch and hands
// it to the next GPU's worker thread (at most kQueue batches wait per GPU), and
// returns.  okm_group_count drains the queues and, with more than one GPU,
// merges the per-GPU tables by key-range owner over RCCL (okm_merge_owned,
// one host thread per GPU, okm_comm_init_all communicators): rank r then owns
// a contiguous key range, so the ranges in rank order are the sorted global
// table (count.rs:106-119).  Only the public C ABI is used.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "okm_internal.h"
#include "orion_kmer_testing.h"
#include "okm_io.h"

namespace {

constexpr size_t kQueue = 2;  // batches waiting per GPU (bounds host memory: the reader's batches are <= 256 MB)

struct Task {
    std::vector<uint8_t> seq;
    std::vector<uint64_t> off;
    uint64_t n = 0;
    int normalized = 0;
};

struct Worker {
    okm_ctx *ctx = nullptr;
    okm_comm *comm = nullptr;
    std::thread th;
    std::deque<Task> q;
    bool busy = false;
    okm_status err = OKM_OK;
    std::string msg;
};

}  // namespace

struct okm_group {
    uint8_t k = 0;
    okm_mode mode = OKM_MODE_COUNT;
    std::vector<Worker> w;
    std::mutex mu;
    std::condition_variable cv;  // queue changes (both directions)
    bool stop = false;
    size_t next = 0;
    bool counted = false;
    uint64_t distinct = 0;
};

namespace {

void worker_loop(okm_group *g, size_t i) {
    Worker &W = g->w[i];
    for (;;) {
        Task t;
        {
            std::unique_lock<std::mutex> lk(g->mu);
            g->cv.wait(lk, [&] { return g->stop || !W.q.empty(); });
            if (W.q.empty()) return;  // stop
            t = std::move(W.q.front());
            W.q.pop_front();
            W.busy = true;
        }
        g->cv.notify_all();
        okm_status s = OKM_OK;
        if (W.err == OKM_OK) s = okm_add_batch(W.ctx, t.seq.data(), t.off.data(), t.n, t.normalized);
        {
            std::lock_guard<std::mutex> lk(g->mu);
            W.busy = false;
            if (s != OKM_OK && W.err == OKM_OK) {
                W.err = s;
                W.msg = okm_last_error();
            }
        }
        g->cv.notify_all();
    }
}

// Waits until every queue is empty and every worker idle; returns the first error.
okm_status drain(okm_group *g) {
    std::unique_lock<std::mutex> lk(g->mu);
    g->cv.wait(lk, [&] {
        for (auto &W : g->w)
            if (!W.q.empty() || W.busy) return false;
        return true;
    });
    for (auto &W : g->w)
        if (W.err != OKM_OK) return okm::fail(W.err, W.msg);
    return OKM_OK;
}

}  // namespace

extern "C" {

okm_status okm_group_create(okm_group **out, uint8_t k, okm_mode mode, int n_gpus, const int *devices,
                            uint64_t distinct_hint) {
    if (!out) return okm::fail(OKM_E_ARG, "okm_group_create: null out");
    *out = nullptr;
    const int avail = okm_device_count();
    if (avail <= 0) return okm::fail(OKM_E_DEVICE, "no HIP device visible (the engine has no CPU fallback)");
    const int n = n_gpus <= 0 ? avail : n_gpus;
    if (n > avail)
        return okm::fail(OKM_E_ARG, "okm_group_create: " + std::to_string(n) + " GPUs asked, " + std::to_string(avail) +
                                        " visible (one context per GPU)");
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) {
        devs[i] = devices ? devices[i] : i;
        if (devs[i] < 0 || devs[i] >= avail)
            return okm::fail(OKM_E_ARG, "okm_group_create: device " + std::to_string(devs[i]) + " of " +
                                            std::to_string(n) + " GPUs asked, " + std::to_string(avail) + " visible");
        for (int j = 0; j < i; ++j)
            if (devs[j] == devs[i])
                return okm::fail(OKM_E_ARG, "okm_group_create: device " + std::to_string(devs[i]) + " named twice");
    }
    okm_group *g = new okm_group();
    g->k = k;
    g->mode = mode;
    g->w.resize(n);
    for (int i = 0; i < n; ++i) {
        okm_status s = okm_create(&g->w[i].ctx, k, mode, devs[i], distinct_hint);
        if (s != OKM_OK) {
            okm_group_destroy(g);
            return s;
        }
    }
    if (n > 1) {
        std::vector<okm_comm *> comms(n, nullptr);
        okm_status s = okm_comm_init_all(comms.data(), n, devs.data());
        if (s != OKM_OK) {
            okm_group_destroy(g);
            return s;
        }
        for (int i = 0; i < n; ++i) g->w[i].comm = comms[i];
    }
    for (int i = 0; i < n; ++i) g->w[i].th = std::thread(worker_loop, g, (size_t)i);
    *out = g;
    return OKM_OK;
}

void okm_group_destroy(okm_group *g) {
    if (!g) return;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        g->stop = true;
    }
    g->cv.notify_all();
    for (auto &W : g->w)
        if (W.th.joinable()) W.th.join();
    for (auto &W : g->w) {
        if (W.comm) okm_comm_destroy(W.comm);
        if (W.ctx) okm_destroy(W.ctx);
    }
    delete g;
}

int okm_group_size(const okm_group *g) { return g ? (int)g->w.size() : 0; }

okm_status okm_group_add_batch(okm_group *g, const uint8_t *seq, const uint64_t *offsets, uint64_t n_records,
                               int normalized) {
    if (!g) return okm::fail(OKM_E_ARG, "null group");
    if (n_records == 0) return OKM_OK;
    if (!offsets || (!seq && offsets[n_records] > offsets[0])) return okm::fail(OKM_E_ARG, "okm_group_add_batch: null buffer");
    Task t;
    const uint64_t base = offsets[0], bytes = offsets[n_records] - base;
    t.seq.assign(seq + base, seq + base + bytes);
    t.off.resize(n_records + 1);
    for (uint64_t r = 0; r <= n_records; ++r) t.off[r] = offsets[r] - base;
    t.n = n_records;
    t.normalized = normalized;
    std::unique_lock<std::mutex> lk(g->mu);
    // the next GPU in turn with room in its queue (back-pressure on the reader)
    size_t pick = g->w.size();
    g->cv.wait(lk, [&] {
        for (size_t j = 0; j < g->w.size(); ++j) {
            const size_t i = (g->next + j) % g->w.size();
            if (g->w[i].err != OKM_OK) {
                pick = i;
                return true;
            }
            if (g->w[i].q.size() < kQueue) {
                pick = i;
                return true;
            }
        }
        return false;
    });
    Worker &W = g->w[pick];
    if (W.err != OKM_OK) return okm::fail(W.err, W.msg);
    g->next = (pick + 1) % g->w.size();
    W.q.push_back(std::move(t));
    g->counted = false;
    lk.unlock();
    g->cv.notify_all();
    return OKM_OK;
}

okm_status okm_group_count(okm_group *g, uint64_t *n_distinct) {
    if (!g) return okm::fail(OKM_E_ARG, "null group");
    okm_status s = drain(g);
    if (s != OKM_OK) return s;
    if (!g->counted) {
        const size_t n = g->w.size();
        std::vector<okm_status> st(n, OKM_OK);
        std::vector<std::string> msg(n);
        std::vector<uint64_t> owned(n, 0);
        auto run = [&](size_t i) {
            Worker &W = g->w[i];
            st[i] = W.comm ? okm_merge_owned(W.ctx, W.comm, W.ctx, &owned[i]) : okm_count(W.ctx, &owned[i]);
            if (st[i] != OKM_OK) msg[i] = okm_last_error();
        };
        if (n == 1) {
            run(0);
        } else {  // one host thread per rank: the collectives of every rank progress together
            std::vector<std::thread> ts;
            for (size_t i = 0; i < n; ++i) ts.emplace_back(run, i);
            for (auto &t : ts) t.join();
        }
        g->distinct = 0;
        for (size_t i = 0; i < n; ++i) {
            if (st[i] != OKM_OK) return okm::fail(st[i], "rank " + std::to_string(i) + ": " + msg[i]);
            g->distinct += owned[i];
        }
        g->counted = true;
    }
    if (n_distinct) *n_distinct = g->distinct;
    return OKM_OK;
}

okm_ctx *okm_group_owner(okm_group *g, int rank) {
    if (!g || rank < 0 || rank >= (int)g->w.size()) return nullptr;
    return g->w[rank].ctx;
}

okm_status okm_group_finish_counts(okm_group *g, uint64_t min_count, uint64_t **keys, uint64_t **counts,
                                   uint64_t *n) {
    if (!g || !keys || !counts || !n) return okm::fail(OKM_E_ARG, "null argument");
    *keys = *counts = nullptr;
    *n = 0;
    okm_status s = okm_group_count(g, nullptr);
    if (s != OKM_OK) return s;
    const size_t P = g->w.size();
    const uint64_t kw = (g->k > 32) ? 2 : 1;
    std::vector<uint64_t> sz(P), off(P + 1, 0);
    for (size_t r = 0; r < P; ++r) {
        if ((s = okm_result_size(g->w[r].ctx, min_count, &sz[r])) != OKM_OK) return s;
        off[r + 1] = off[r] + sz[r];
    }
    const uint64_t total = off[P];
    uint64_t *K = (uint64_t *)malloc(std::max<uint64_t>(total, 1) * 8 * kw);
    uint64_t *C = (uint64_t *)malloc(std::max<uint64_t>(total, 1) * 8);
    if (!K || !C) {
        free(K);
        free(C);
        return okm::fail(OKM_E_NOMEM, "okm_group_finish_counts: host allocation failed");
    }
    // ranges in rank order = the sorted global table; ranks copy out concurrently
    std::vector<okm_status> st(P, OKM_OK);
    std::vector<std::string> msg(P);
    auto fetch = [&](size_t r) {
        uint64_t got = 0;
        st[r] = okm_fetch_counts(g->w[r].ctx, min_count, K + off[r] * kw, C + off[r], sz[r], &got, 0);
        if (st[r] != OKM_OK) msg[r] = okm_last_error();
    };
    std::vector<std::thread> ts;
    for (size_t r = 0; r < P; ++r) ts.emplace_back(fetch, r);
    for (auto &t : ts) t.join();
    for (size_t r = 0; r < P; ++r)
        if (st[r] != OKM_OK) {
            free(K);
            free(C);
            return okm::fail(st[r], msg[r]);
        }
    *keys = K;
    *counts = C;
    *n = total;
    return OKM_OK;
}

// count.rs:106-137 straight from the device: every owner's range (rank
// order = the sorted global table) is copied off the GPU in chunks into two
// page-locked buffers by a copy thread while the host threads filter, format
// and write the previous chunk (okm::write_counts_tsv_chunks), so the PCIe
// copy hides behind the TSV work and no table-sized host array is touched.
okm_status okm_group_write_counts_tsv(okm_group *g, const char *path, uint64_t min_count, uint64_t *n_lines) {
    if (!g || !path) return okm::fail(OKM_E_ARG, "null argument");
    okm_status s = okm_group_count(g, nullptr);
    if (s != OKM_OK) return s;
    const uint64_t kw = (g->k > 32) ? 2 : 1;
    struct Chunk {
        const uint64_t *k, *c;
        uint64_t n;
        int device;  // the owning GPU: the copy runs on its device, not device 0's
        bool host;   // a table count_spilled left in host memory
    };
    std::vector<Chunk> chunks;
    uint64_t per = uint64_t(1) << 24;  // entries per chunk (256 MB of keys + counts at k <= 32)
    if (const int64_t e = okm::test_knob(OKM_TEST_TSV_CHUNK); e > 0) per = std::max<uint64_t>(1024, (uint64_t)e);
    for (auto &W : g->w) {
        const uint64_t *dk = nullptr, *dc = nullptr;
        uint64_t n = 0;
        bool host = false;
        if ((s = okm::result_view(W.ctx, &dk, &dc, &n, &host)) != OKM_OK) return s;
        for (uint64_t o = 0; o < n; o += per)
            chunks.push_back({dk + o * kw, dc + o, std::min(per, n - o), okm::ctx_device(W.ctx), host});
    }
    uint64_t cap = 0;
    for (auto &c : chunks) cap = std::max(cap, c.n);
    struct Slot {
        uint64_t *k = nullptr, *c = nullptr;
        long chunk = -1;  // chunk held (ready), -1: free
    } slot[2];
    const size_t kbytes = std::max<uint64_t>(cap, 1) * kw * 8, cbytes = std::max<uint64_t>(cap, 1) * 8;
    for (auto &sl : slot) {
        sl.k = (uint64_t *)okm::host_pinned_alloc(kbytes);
        sl.c = (uint64_t *)okm::host_pinned_alloc(cbytes);
    }
    auto release = [&]() {
        for (auto &sl : slot) {
            okm::host_pinned_free(sl.k);
            okm::host_pinned_free(sl.c);
        }
    };
    if (!slot[0].k || !slot[0].c || !slot[1].k || !slot[1].c) {
        release();
        return okm::fail(OKM_E_NOMEM, "okm_group_write_counts_tsv: pinned host buffers");
    }
    std::mutex mu;
    std::condition_variable cv;
    bool stop = false;
    okm_status copy_st = OKM_OK;
    std::string copy_msg;
    size_t consumed = 0;  // chunks [0, consumed) are done with: their slots may be refilled
    std::thread copier([&]() {
        for (size_t i = 0; i < chunks.size(); ++i) {
            Slot &sl = slot[i % 2];
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || i < consumed + 2; });
                if (stop) return;
            }
            okm_status st = OKM_OK;
            if (chunks[i].host) {
                memcpy(sl.k, chunks[i].k, chunks[i].n * kw * 8);
                memcpy(sl.c, chunks[i].c, chunks[i].n * 8);
            } else {
                st = okm::memcpy_d2h_on(chunks[i].device, sl.k, chunks[i].k, chunks[i].n * kw * 8);
                if (st == OKM_OK) st = okm::memcpy_d2h_on(chunks[i].device, sl.c, chunks[i].c, chunks[i].n * 8);
            }
            std::lock_guard<std::mutex> lk(mu);
            if (st != OKM_OK) {
                copy_st = st;
                copy_msg = okm_last_error();
                stop = true;
            } else {
                sl.chunk = (long)i;
            }
            cv.notify_all();
            if (st != OKM_OK) return;
        }
    });
    s = okm::write_counts_tsv_chunks(
        path, g->k, min_count, chunks.size(),
        [&](size_t i, const uint64_t **kp, const uint64_t **cp, uint64_t *np) -> okm_status {
            std::unique_lock<std::mutex> lk(mu);
            consumed = i;  // chunk i - 1 is written: its slot may take chunk i + 1
            cv.notify_all();
            cv.wait(lk, [&] { return stop || slot[i % 2].chunk == (long)i; });
            if (slot[i % 2].chunk != (long)i) return okm::fail(copy_st != OKM_OK ? copy_st : OKM_E_DEVICE, copy_msg);
            *kp = slot[i % 2].k;
            *cp = slot[i % 2].c;
            *np = chunks[i].n;
            return OKM_OK;
        },
        n_lines);
    {
        std::lock_guard<std::mutex> lk(mu);
        stop = true;
        cv.notify_all();
    }
    copier.join();
    release();
    return s;
}

}  // extern "C"
