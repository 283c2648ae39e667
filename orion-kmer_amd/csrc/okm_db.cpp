// okm_db.cpp — KmerDbV2 (db_types.rs:7-14) in bincode 1.3's default encoding,
// the format `build` writes (build.rs:141-146) and `compare`/`query`/`classify`
// read (utils.rs:37-55):
//   u8 k
//   u64 n_refs                            HashMap<String, HashSet<u64>> length
//   n_refs × { u64 len, len bytes UTF-8,  String
//              u64 n, n × u64 }           HashSet<u64>
// all little-endian, fixed-width integers.  The reference's HashMap/HashSet
// iteration order is random (RandomState), so bytes are not reproducible there
// either; we write references in insertion order and keys sorted ascending.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "okm_internal.h"
#include "okm_io.h"

using namespace okm;

struct okm_db {
    uint8_t k = 0;
    std::vector<std::string> names;
    std::vector<std::vector<uint64_t>> keys;
};

static void put_u64(Bytes &b, uint64_t v) {
    for (int i = 0; i < 8; ++i) b.push_back((uint8_t)(v >> (8 * i)));
}

extern "C" {

okm_status okm_db_new(okm_db **out, uint8_t k) {
    if (!out) return fail(OKM_E_ARG, "null out");
    *out = new okm_db();
    (*out)->k = k;
    return OKM_OK;
}

okm_status okm_db_add_reference(okm_db *db, const char *name, const uint64_t *keys, uint64_t n) {
    if (!db || !name || (!keys && n)) return fail(OKM_E_ARG, "null argument");
    std::vector<uint64_t> v(keys, keys + n);
    for (size_t i = 0; i < db->names.size(); ++i) {
        if (db->names[i] == name) {  // db_types.rs:38-40: insert overwrites
            db->keys[i].swap(v);
            return OKM_OK;
        }
    }
    db->names.emplace_back(name);
    db->keys.push_back(std::move(v));
    return OKM_OK;
}

okm_status okm_db_write(const okm_db *db, const char *path) {
    if (!db || !path) return fail(OKM_E_ARG, "null argument");
    OutWriter w;
    okm_status s = w.open(path);
    if (s != OKM_OK) return s;
    Bytes b;
    b.push_back(db->k);
    put_u64(b, db->names.size());
    for (size_t i = 0; i < db->names.size(); ++i) {
        put_u64(b, db->names[i].size());
        b.insert(b.end(), db->names[i].begin(), db->names[i].end());
        put_u64(b, db->keys[i].size());
        const size_t at = b.size();
        b.resize(at + 8 * db->keys[i].size());
        memcpy(b.data() + at, db->keys[i].data(), 8 * db->keys[i].size());  // x86-64: little-endian
        if (b.size() > (64u << 20)) {
            s = w.write(b.data(), b.size());
            if (s != OKM_OK) return s;
            b.clear();
        }
    }
    s = w.write(b.data(), b.size());
    if (s != OKM_OK) return s;
    return w.close();
}

okm_status okm_db_read(okm_db **out, const char *path) {
    if (!out || !path) return fail(OKM_E_ARG, "null argument");
    *out = nullptr;
    Bytes d;
    okm_status s = read_whole_file(path, d);
    if (s != OKM_OK) return s;
    if (decompress_by_extension(path, d) != OKM_OK) return fail(OKM_E_FORMAT, okm_last_error());
    size_t p = 0;
    auto need = [&](size_t n) { return p + n <= d.size(); };
    auto get_u64 = [&](uint64_t &v) {
        if (!need(8)) return false;
        v = 0;
        for (int i = 0; i < 8; ++i) v |= (uint64_t)d[p + i] << (8 * i);
        p += 8;
        return true;
    };
    okm_db *db = new okm_db();
    bool ok = need(1);
    if (ok) db->k = d[p++];
    uint64_t nrefs = 0;
    ok = ok && get_u64(nrefs);
    for (uint64_t r = 0; ok && r < nrefs; ++r) {
        uint64_t len = 0, n = 0;
        ok = get_u64(len) && need(len);
        if (!ok) break;
        std::string name((const char *)d.data() + p, len);
        p += len;
        ok = get_u64(n) && n <= (d.size() - p) / 8;
        if (!ok) break;
        std::vector<uint64_t> v(n);
        memcpy(v.data(), d.data() + p, 8 * n);
        p += 8 * n;
        db->names.push_back(std::move(name));
        db->keys.push_back(std::move(v));
    }
    if (!ok) {
        delete db;
        return fail(OKM_E_FORMAT, "truncated or malformed KmerDbV2");
    }
    *out = db;
    return OKM_OK;
}

uint8_t okm_db_k(const okm_db *db) { return db ? db->k : 0; }
uint64_t okm_db_num_references(const okm_db *db) { return db ? db->names.size() : 0; }

okm_status okm_db_reference(const okm_db *db, uint64_t i, const char **name, const uint64_t **keys, uint64_t *n) {
    if (!db || i >= db->names.size()) return fail(OKM_E_ARG, "reference index out of range");
    if (name) *name = db->names[i].c_str();
    if (keys) *keys = db->keys[i].data();
    if (n) *n = db->keys[i].size();
    return OKM_OK;
}

void okm_db_free(okm_db *db) { delete db; }

}  // extern "C"
