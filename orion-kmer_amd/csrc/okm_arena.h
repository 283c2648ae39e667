// okm_arena.h — a counting context's device memory arena.
//
// One reserved virtual address range per context (2x the device's HBM), with
// physical memory mapped into it in fixed chunks (hipMemCreate / hipMemMap; 1 GiB)
// as allocations need them.  Allocations are best-fit ranges of the address
// space; freed ranges coalesce with their neighbours, so a 9 GB request is
// served by any free 9 GB stretch, whatever sizes were freed to make it.
// The physical chunks of freed ranges stay mapped (cached) and are unmapped
// only under memory pressure (the pools' soft cap, OKM_HBM_CAP) or trim.
//
// Why: a context that works near the HBM cap (BASELINE configs[2] on one GPU
// folds batches into sorted tables; the N>1 merge adds an owner table and the
// communicator's buffers) needs blocks of many multi-GB sizes in turn.  A
// cache of whole hipMalloc blocks serves a request only from a block of about
// its size, so near the cap it freed and re-mapped tens of GB per count —
// 0.4-1.4 s host stalls per phase.  Here no count after the
// first maps anything.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <vector>

namespace okm {

struct VmmArena {
    int device = -1;
    char *base = nullptr;
    size_t reserved = 0;  // bytes of address space
    size_t chunk = 0;     // bytes per physical chunk
    struct Chunk {
        hipMemGenericAllocationHandle_t h{};
        bool mapped = false;
        uint32_t users = 0;  // live ranges touching the chunk
    };
    std::vector<Chunk> chunks;
    std::map<size_t, size_t> free_off;      // offset -> length (coalesced)
    std::multimap<size_t, size_t> free_sz;  // length -> offset (best fit)
    std::map<size_t, size_t> live;          // offset -> length
    size_t mapped = 0;                      // bytes of mapped chunks
    size_t in_use = 0;                      // bytes of live ranges

    static size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

    hipMemAllocationProp prop() const {
        hipMemAllocationProp p{};
        p.type = hipMemAllocationTypePinned;
        p.location.type = hipMemLocationTypeDevice;
        p.location.id = device;
        return p;
    }

    // Reserve the address range; false (and nothing held) when the device or
    // runtime has no virtual memory management.
    bool init(int dev, size_t chunk_bytes) {
        device = dev;
        int vmm = 0;
        if (hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, dev) != hipSuccess ||
            !vmm) {
            (void)hipGetLastError();
            return false;
        }
        size_t gran = 0;
        hipMemAllocationProp p = prop();
        if (hipMemGetAllocationGranularity(&gran, &p, hipMemAllocationGranularityRecommended) != hipSuccess ||
            gran == 0) {
            (void)hipGetLastError();
            return false;
        }
        chunk = round_up(std::max(chunk_bytes, gran), gran);
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess || tot == 0) {
            (void)hipGetLastError();
            return false;
        }
        reserved = round_up(2 * tot, chunk);
        void *va = nullptr;
        if (hipMemAddressReserve(&va, reserved, chunk, nullptr, 0) != hipSuccess || !va) {
            (void)hipGetLastError();
            reserved = 0;
            return false;
        }
        base = static_cast<char *>(va);
        chunks.assign(reserved / chunk, Chunk{});
        free_off[0] = reserved;
        free_sz.emplace(reserved, 0);
        return true;
    }

    void erase_free(size_t off, size_t len) {
        free_off.erase(off);
        auto r = free_sz.equal_range(len);
        for (auto it = r.first; it != r.second; ++it)
            if (it->second == off) {
                free_sz.erase(it);
                return;
            }
    }
    void add_free(size_t off, size_t len) {
        // coalesce with the ranges on either side
        auto next = free_off.lower_bound(off);
        if (next != free_off.end() && next->first == off + len) {
            len += next->second;
            erase_free(next->first, next->second);
        }
        auto prev = free_off.lower_bound(off);
        if (prev != free_off.begin()) {
            --prev;
            if (prev->first + prev->second == off) {
                off = prev->first;
                len += prev->second;
                erase_free(prev->first, prev->second);
            }
        }
        free_off[off] = len;
        free_sz.emplace(len, off);
    }

    // Best-fit range of `bytes` (a multiple of 256); ~0 when the address space is exhausted.
    size_t take(size_t bytes) {
        auto it = free_sz.lower_bound(bytes);
        if (it == free_sz.end()) return ~size_t(0);
        const size_t len = it->first, off = it->second;
        erase_free(off, len);
        if (len > bytes) add_free(off + bytes, len - bytes);
        live[off] = bytes;
        in_use += bytes;
        return off;
    }
    void give_back(size_t off) {
        auto it = live.find(off);
        if (it == live.end()) return;
        const size_t len = it->second;
        live.erase(it);
        in_use -= len;
        add_free(off, len);
    }
    // Keep the first `bytes` of a live range and give back its tail (no copy);
    // the chunks past the new end lose this range as a user.
    void shrink(size_t off, size_t bytes) {
        auto it = live.find(off);
        if (it == live.end() || bytes >= it->second) return;
        const size_t len = it->second;
        for (size_t i = last_chunk(off, bytes) + 1; i <= last_chunk(off, len); ++i) chunks[i].users--;
        it->second = bytes;
        in_use -= len - bytes;
        add_free(off + bytes, len - bytes);
    }
    size_t first_chunk(size_t off) const { return off / chunk; }
    size_t last_chunk(size_t off, size_t len) const { return (off + len - 1) / chunk; }

    hipError_t map_chunk(size_t i) {
        Chunk &c = chunks[i];
        hipMemAllocationProp p = prop();
        hipError_t e = hipMemCreate(&c.h, chunk, &p, 0);
        if (e != hipSuccess) return e;
        e = hipMemMap(base + i * chunk, chunk, 0, c.h, 0);
        if (e != hipSuccess) {
            (void)hipMemRelease(c.h);
            return e;
        }
        hipMemAccessDesc d{};
        d.location.type = hipMemLocationTypeDevice;
        d.location.id = device;
        d.flags = hipMemAccessFlagsProtReadWrite;
        e = hipMemSetAccess(base + i * chunk, chunk, &d, 1);
        if (e != hipSuccess) {
            (void)hipMemUnmap(base + i * chunk, chunk);
            (void)hipMemRelease(c.h);
            return e;
        }
        c.mapped = true;
        mapped += chunk;
        return hipSuccess;
    }
    void unmap_chunk(size_t i) {
        Chunk &c = chunks[i];
        if (!c.mapped) return;
        (void)hipMemUnmap(base + i * chunk, chunk);
        (void)hipMemRelease(c.h);
        c.mapped = false;
        mapped -= chunk;
    }
    // Bytes of mapped chunks no live range touches.
    size_t idle() const {
        size_t b = 0;
        for (const Chunk &c : chunks)
            if (c.mapped && !c.users) b += chunk;
        return b;
    }
    // Unmap idle chunks until `want` bytes came back (everything idle when
    // want == ~0).  The caller has synchronised the device: an unmapped chunk
    // must not be in use by a kernel still in flight.
    size_t unmap_idle(size_t want) {
        size_t got = 0;
        for (size_t i = chunks.size(); i-- > 0 && got < want;)
            if (chunks[i].mapped && !chunks[i].users) {
                unmap_chunk(i);
                got += chunk;
            }
        return got;
    }
    void release() {
        if (!base) return;
        (void)hipDeviceSynchronize();
        for (size_t i = 0; i < chunks.size(); ++i) unmap_chunk(i);
        (void)hipMemAddressFree(base, reserved);
        (void)hipGetLastError();
        base = nullptr;
        chunks.clear();
        free_off.clear();
        free_sz.clear();
        live.clear();
        mapped = in_use = 0;
    }
};

}  // namespace okm
