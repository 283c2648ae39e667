// Host-side check of the SWAR window helpers of okm_scan.h (the same
// __host__ __device__ code the extraction and query kernels run): every window
// of random byte buffers against a per-window restatement of kmer.rs:12-106
// (seq_to_u64 + reverse_complement + canonical, O(k) per window), for k in
// 1..64, normalize-mode validity (U valid, = T) and raw query-mode validity.
// Built and run by tests/test_scan_codes.py; prints "ok" or the first mismatch.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "okm_scan.h"

using namespace okm;

static int code_of(unsigned char c, bool raw, bool *ok) {
    switch (c) {
    case 'A': case 'a': *ok = true; return 0;
    case 'C': case 'c': *ok = true; return 1;
    case 'G': case 'g': *ok = true; return 2;
    case 'T': case 't': *ok = true; return 3;
    case 'U': case 'u': *ok = !raw; return 3;
    default: *ok = false; return 0;
    }
}

// kmer.rs:37-106 on bytes [j, j+k): canonical value as (hi, lo), validity
static bool naive(const unsigned char *b, int j, int k, bool raw, unsigned long long *hi, unsigned long long *lo) {
    unsigned __int128 f = 0, r = 0;
    bool valid = true;
    for (int i = 0; i < k; ++i) {
        bool ok;
        int c = code_of(b[j + i], raw, &ok);
        valid &= ok;
        f = (f << 2) | (unsigned)c;
        r |= (unsigned __int128)(c ^ 3) << (2 * i);
    }
    unsigned __int128 m = f < r ? f : r;
    *hi = (unsigned long long)(m >> 64);
    *lo = (unsigned long long)m;
    return valid;
}

template <int NP, bool RAW>
static int check(const unsigned char *buf, int seg, int kmax) {
    uint32_t w[NP * 4];
    memcpy(w, buf, sizeof(w));
    Codes<NP> c;
    make_codes<NP, RAW>(w, c);
    for (int k = 1; k <= kmax; ++k) {
        for (int j = 0; j < seg && j + k <= NP * 16; ++j) {
            unsigned long long hi, lo;
            const bool nv = naive(buf, j, k, RAW, &hi, &lo);
            bool v;
            if (k <= 32) {
                const uint64_t key = window_key(c, j, (uint32_t)k, &v);
                if (v != nv || (v && (key != lo || hi != 0))) {
                    printf("mismatch k=%d j=%d raw=%d valid %d/%d key %llx/%llx\n", k, j, RAW, v, nv,
                           (unsigned long long)key, lo);
                    return 1;
                }
            } else {
                const K128 key = window_key128(c, j, (uint32_t)k, &v);
                if (v != nv || (v && (key.lo != lo || key.hi != hi))) {
                    printf("mismatch128 k=%d j=%d valid %d/%d key %llx:%llx/%llx:%llx\n", k, j, v, nv, key.hi,
                           key.lo, hi, lo);
                    return 1;
                }
            }
        }
    }
    return 0;
}

// invalid_windows (scan_words' all-windows validity mask) against the per-window test
template <int NP, int SEG, bool RAW>
static int check_inv(const unsigned char *buf) {
    uint32_t w[NP * 4];
    memcpy(w, buf, sizeof(w));
    Codes<NP> c;
    make_codes<NP, RAW>(w, c);
    for (int k = 1; k <= 32; ++k) {
        const uint32_t inv = invalid_windows<SEG, NP>(c, (uint32_t)k);
        for (int j = 0; j < SEG; ++j) {
            unsigned long long hi, lo;
            const bool nv = naive(buf, j, k, RAW, &hi, &lo);
            if ((((inv >> j) & 1u) == 0) != nv) {
                printf("invalid_windows k=%d j=%d seg=%d raw=%d: mask says %d, naive %d\n", k, j, SEG, RAW,
                       (int)(((inv >> j) & 1u) == 0), nv);
                return 1;
            }
        }
    }
    return 0;
}

int main() {
    srand(12345);
    static const char alpha[] = "ACGTACGTACGTACGTacgtUuNn\n-.~ RYK";
    unsigned char buf[160];
    for (int it = 0; it < 3000; ++it) {
        const int mode = it % 4;  // mostly valid / mixed / all upper / random bytes
        for (int i = 0; i < 160; ++i) {
            unsigned char ch;
            if (mode == 0) ch = "ACGT"[rand() & 3];
            else if (mode == 1) ch = alpha[rand() % (int)(sizeof(alpha) - 1)];
            else if (mode == 2) ch = (rand() % 50) ? "ACGTacgt"[rand() & 7] : "NU\nu"[rand() & 3];
            else ch = (unsigned char)rand();
            buf[i] = ch;
        }
        if (check<3, false>(buf, 16, 32) || check<3, true>(buf, 16, 32)) return 1;   // scatter / query
        if (check_inv<3, 16, false>(buf) || check_inv<3, 16, true>(buf) || check_inv<4, 32, false>(buf)) return 1;
        if (check<6, false>(buf, 64, 32)) return 1;                                   // hist
        if (check<5, false>(buf, 16, 64) || check<8, false>(buf, 64, 64)) return 1;   // wide
    }
    printf("ok\n");
    return 0;
}
