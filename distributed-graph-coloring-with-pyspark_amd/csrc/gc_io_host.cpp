// gc_io_host.cpp -- graph files for the drop-in CLI.
//
// 1. The reference's JSON graph (graph.py:15-28 deserialize_graph, node.py:8-13 to_dict):
//    a list of {"id", "neighbors", "color"} objects.  gc_json_read_graph parses it in one
//    pass over an mmap of the file and resolves neighbour ids to FILE POSITIONS exactly as
//    graph.py:23-26 does: node_dict = {id: node} keeps the LAST node of a repeated id, the
//    input colour is ignored (graph.py:20), and the first neighbour id (file order) that is
//    not a node id is a KeyError (GC_EKEY, gc_last_error() = the id, which the Python host
//    re-raises as KeyError(id) -> "Error loading graph: <id>", coloring.py:179-181).
//    The native reader is exact on the files it accepts: integer ids that fit int64,
//    neighbour lists of such integers, keys without escapes, strict JSON elsewhere.  Any
//    other input (string / float / boolean ids, non-list neighbours, missing keys, NaN,
//    non-ASCII text, malformed JSON, ...) returns GC_EUNSUPPORTED without guessing, and the
//    host re-reads that file with Python's json + graph.py's own linking rules, which raise
//    the reference's exact exception.
// 2. json.dump(indent=4) writers for the colouring output (coloring.py:238-241) and the
//    serialised graph (graph.py:10-12): byte-identical to Python's encoder for int ids.
// 3. A binary CSR file (.gcsr) for graphs too big for JSON (C2-C5: 1.8 MB of JSON per 10^4
//    vertices).  Layout (little endian):
//      0  char[8] "GCSR\0\0\0\1"   8 int64 n   16 int64 nnz   24 uint32 flags
//      28 uint32 has_ids           32 int64 row_ptr[n+1]      then int32 col[nnz]
//      pad to 8 bytes              then int64 ids[n] when has_ids
//    Reading checks the header against the file size, row_ptr monotone from 0 to nnz and
//    every col entry in [0, n).
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "gcolor.h"

void gc_set_error(const char* fmt, ...);

namespace {

const char kMagic[8] = {'G', 'C', 'S', 'R', 0, 0, 0, 1};

struct Mapped {
    const char* p = nullptr;
    size_t len = 0;
    int fd = -1;
    ~Mapped() {
        if (p && len) munmap((void*)p, len);
        if (fd >= 0) close(fd);
    }
    int open_file(const char* path) {
        fd = ::open(path, O_RDONLY);
        if (fd < 0) {
            gc_set_error("[Errno %d] %s: '%s'", errno, strerror(errno), path);
            return GC_EIO;
        }
        struct stat sb;
        if (fstat(fd, &sb) != 0) {
            gc_set_error("fstat(%s): %s", path, strerror(errno));
            return GC_EIO;
        }
        len = (size_t)sb.st_size;
        if (len == 0) return GC_OK;
        void* m = mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) {
            gc_set_error("mmap(%s): %s", path, strerror(errno));
            p = nullptr;
            len = 0;
            return GC_EIO;
        }
        madvise(m, len, MADV_SEQUENTIAL);
        p = (const char*)m;
        return GC_OK;
    }
};

// Strict JSON scanner over [p, e).  Every "unsupported" answer makes the whole read
// GC_EUNSUPPORTED (the Python host then applies json.load's and graph.py's own rules).
struct Scan {
    const char* p;
    const char* e;
    bool bad = false;

    void ws() {
        while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
    }
    bool lit(char c) {
        ws();
        if (p < e && *p == c) {
            ++p;
            return true;
        }
        return false;
    }
    bool peek(char c) {
        ws();
        return p < e && *p == c;
    }
    // integer token (JSON grammar, no fraction/exponent) that fits int64
    bool integer(int64_t* out) {
        ws();
        const char* s = p;
        bool neg = false;
        if (s < e && *s == '-') {
            neg = true;
            ++s;
        }
        if (s >= e || *s < '0' || *s > '9') return false;
        if (*s == '0' && s + 1 < e && s[1] >= '0' && s[1] <= '9') return false;  // leading zero: invalid JSON
        unsigned __int128 v = 0;
        const char* d0 = s;
        while (s < e && *s >= '0' && *s <= '9') {
            v = v * 10 + (unsigned)(*s - '0');
            if (v > ((unsigned __int128)1 << 63)) return false;
            ++s;
            if (s - d0 > 20) return false;
        }
        if (s < e && (*s == '.' || *s == 'e' || *s == 'E')) return false;  // a float
        if (!neg && v > (unsigned __int128)INT64_MAX) return false;
        *out = neg ? (int64_t)(0 - (uint64_t)v) : (int64_t)v;
        p = s;
        return true;
    }
    // a key without escapes and ASCII only; returns [k, klen)
    bool key(const char** k, size_t* klen) {
        ws();
        if (p >= e || *p != '"') return false;
        const char* s = ++p;
        while (p < e && *p != '"') {
            unsigned char c = (unsigned char)*p;
            if (c == '\\' || c < 0x20 || c >= 0x80) return false;
            ++p;
        }
        if (p >= e) return false;
        *k = s;
        *klen = (size_t)(p - s);
        ++p;
        return lit(':');
    }
    bool skip_string() {  // at '"'
        ++p;
        while (p < e) {
            unsigned char c = (unsigned char)*p++;
            if (c == '"') return true;
            if (c < 0x20 || c >= 0x80) return false;
            if (c == '\\') {
                if (p >= e) return false;
                char x = *p++;
                if (x == 'u') {
                    for (int i = 0; i < 4; ++i, ++p) {
                        if (p >= e) return false;
                        char h = *p;
                        if (!((h >= '0' && h <= '9') || (h >= 'a' && h <= 'f') || (h >= 'A' && h <= 'F')))
                            return false;
                    }
                } else if (!strchr("\"\\/bfnrt", x) || x == 0) {
                    return false;
                }
            }
        }
        return false;
    }
    bool skip_number() {
        const char* s = p;
        if (s < e && *s == '-') ++s;
        if (s >= e || *s < '0' || *s > '9') return false;
        if (*s == '0') {
            ++s;
        } else {
            while (s < e && *s >= '0' && *s <= '9') ++s;
        }
        if (s < e && *s == '.') {
            ++s;
            if (s >= e || *s < '0' || *s > '9') return false;
            while (s < e && *s >= '0' && *s <= '9') ++s;
        }
        if (s < e && (*s == 'e' || *s == 'E')) {
            ++s;
            if (s < e && (*s == '+' || *s == '-')) ++s;
            if (s >= e || *s < '0' || *s > '9') return false;
            while (s < e && *s >= '0' && *s <= '9') ++s;
        }
        p = s;
        return true;
    }
    bool word(const char* w) {
        size_t l = strlen(w);
        if ((size_t)(e - p) < l || memcmp(p, w, l) != 0) return false;
        p += l;
        return true;
    }
    bool skip_value(int depth = 0) {
        if (depth > 64) return false;
        ws();
        if (p >= e) return false;
        char c = *p;
        if (c == '"') return skip_string();
        if (c == '-' || (c >= '0' && c <= '9')) return skip_number();
        if (c == 't') return word("true");
        if (c == 'f') return word("false");
        if (c == 'n') return word("null");
        if (c == '[') {
            ++p;
            if (lit(']')) return true;
            for (;;) {
                if (!skip_value(depth + 1)) return false;
                if (lit(',')) continue;
                return lit(']');
            }
        }
        if (c == '{') {
            ++p;
            if (lit('}')) return true;
            for (;;) {
                ws();
                if (p >= e || *p != '"' || !skip_string() || !lit(':') || !skip_value(depth + 1)) return false;
                if (lit(',')) continue;
                return lit('}');
            }
        }
        return false;  // NaN / Infinity and anything else: left to Python
    }
};

// open-addressing id -> position map; insertion in file order, a repeated id keeps the
// last position (graph.py:23, a dict comprehension)
struct IdMap {
    std::vector<int64_t> keys;
    std::vector<int32_t> vals;  // -1 = empty
    size_t mask = 0;
    static uint64_t h(int64_t k) {
        uint64_t z = (uint64_t)k * 0x9E3779B97F4A7C15ull;
        return z ^ (z >> 29);
    }
    void init(size_t n) {
        size_t cap = 16;
        while (cap < 2 * n + 16) cap <<= 1;
        keys.assign(cap, 0);
        vals.assign(cap, -1);
        mask = cap - 1;
    }
    void put(int64_t k, int32_t v) {
        size_t i = h(k) & mask;
        while (vals[i] >= 0 && keys[i] != k) i = (i + 1) & mask;
        keys[i] = k;
        vals[i] = v;
    }
    int32_t get(int64_t k) const {
        size_t i = h(k) & mask;
        while (vals[i] >= 0) {
            if (keys[i] == k) return vals[i];
            i = (i + 1) & mask;
        }
        return -1;
    }
};

gc_csr* csr_new(int64_t n, int64_t nnz, bool with_ids) {
    gc_csr* c = (gc_csr*)calloc(1, sizeof(gc_csr));
    if (!c) return nullptr;
    c->n = n;
    c->nnz = nnz;
    c->row_ptr = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
    c->col = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nnz > 0 ? nnz : 1));
    c->ids = with_ids ? (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1)) : nullptr;
    if (!c->row_ptr || !c->col || (with_ids && !c->ids)) {
        gc_csr_free(c);
        return nullptr;
    }
    return c;
}

// buffered writer with a fast integer formatter
struct Out {
    FILE* f = nullptr;
    std::vector<char> buf;
    size_t used = 0;
    bool err = false;
    explicit Out(FILE* ff) : f(ff), buf(1 << 22) {}
    void flush() {
        if (used && fwrite(buf.data(), 1, used, f) != used) err = true;
        used = 0;
    }
    void room(size_t k) {
        if (used + k > buf.size()) flush();
    }
    void put(const char* s, size_t l) {
        room(l);
        memcpy(buf.data() + used, s, l);
        used += l;
    }
    void puts_(const char* s) { put(s, strlen(s)); }
    void num(int64_t v) {
        room(24);
        char tmp[24];
        int i = 0;
        uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
        do {
            tmp[i++] = (char)('0' + u % 10);
            u /= 10;
        } while (u);
        if (v < 0) buf[used++] = '-';
        while (i) buf[used++] = tmp[--i];
    }
};

FILE* open_out(const char* path) {
    FILE* f = fopen(path, "wb");
    if (!f) gc_set_error("[Errno %d] %s: '%s'", errno, strerror(errno), path);
    return f;
}

int close_out(Out& o, const char* path) {
    o.flush();
    int rc = fclose(o.f);
    if (o.err || rc != 0) {
        gc_set_error("write to %s failed: %s", path, strerror(errno));
        return GC_EIO;
    }
    return GC_OK;
}

}  // namespace

extern "C" void gc_csr_free(gc_csr* c) {
    if (!c) return;
    free(c->row_ptr);
    free(c->col);
    free(c->ids);
    free(c);
}

extern "C" int gc_json_read_graph(const char* path, gc_csr** out) {
    if (!path || !out) {
        gc_set_error("gc_json_read_graph: null argument");
        return GC_EINVAL;
    }
    *out = nullptr;
    Mapped m;
    int rc = m.open_file(path);
    if (rc) return rc;
    Scan s{m.p, m.p + m.len};
    auto unsupported = [&](const char* why) {
        gc_set_error("native JSON reader: %s at byte %lld", why, (long long)(s.p - m.p));
        return GC_EUNSUPPORTED;
    };
    if (m.len == 0) return unsupported("empty file");
    if (!s.lit('[')) return unsupported("top level is not a list");
    std::vector<int64_t> ids;
    std::vector<int64_t> rp(1, 0);
    std::vector<int64_t> nb;  // neighbour ids, resolved below
    if (!s.lit(']')) {
        for (;;) {
            if (!s.lit('{')) return unsupported("list element is not an object");
            bool have_id = false, have_nb = false;
            int64_t id = 0;
            if (!s.lit('}')) {
                for (;;) {
                    const char* k;
                    size_t kl;
                    if (!s.key(&k, &kl)) return unsupported("key");
                    if (kl == 2 && memcmp(k, "id", 2) == 0) {
                        if (have_id || !s.integer(&id)) return unsupported("id");
                        have_id = true;
                    } else if (kl == 9 && memcmp(k, "neighbors", 9) == 0) {
                        if (have_nb || !s.lit('[')) return unsupported("neighbors");
                        have_nb = true;
                        if (!s.lit(']')) {
                            for (;;) {
                                int64_t u;
                                if (!s.integer(&u)) return unsupported("neighbour id");
                                nb.push_back(u);
                                if (s.lit(',')) continue;
                                if (s.lit(']')) break;
                                return unsupported("neighbour list");
                            }
                        }
                    } else if (!s.skip_value()) {
                        return unsupported("value");
                    }
                    if (s.lit(',')) continue;
                    if (s.lit('}')) break;
                    return unsupported("object");
                }
            }
            if (!have_id || !have_nb) return unsupported("missing id or neighbors");
            ids.push_back(id);
            rp.push_back((int64_t)nb.size());
            if (s.lit(',')) continue;
            if (s.lit(']')) break;
            return unsupported("list");
        }
    }
    s.ws();
    if (s.p != s.e) return unsupported("extra data");
    const int64_t n = (int64_t)ids.size(), nnz = (int64_t)nb.size();
    if (n > INT32_MAX) return unsupported("more than 2^31-1 nodes");
    gc_csr* c = csr_new(n, nnz, true);
    if (!c) {
        gc_set_error("gc_json_read_graph: out of host memory");
        return GC_ENOMEM;
    }
    memcpy(c->row_ptr, rp.data(), sizeof(int64_t) * (size_t)(n + 1));
    if (n) memcpy(c->ids, ids.data(), sizeof(int64_t) * (size_t)n);  // (an empty vector's data() may be null)
    bool identity = true;  // ids == 0..n-1 in order: positions are the ids
    for (int64_t i = 0; i < n && identity; ++i) identity = ids[(size_t)i] == i;
    IdMap map;
    if (!identity) {
        map.init((size_t)n);
        for (int64_t i = 0; i < n; ++i) map.put(ids[(size_t)i], (int32_t)i);
    }
    for (int64_t e = 0; e < nnz; ++e) {
        const int64_t u = nb[(size_t)e];
        int32_t pos = identity ? (u >= 0 && u < n ? (int32_t)u : -1) : map.get(u);
        if (pos < 0) {  // graph.py:25: node_dict[neighbor_id] -> KeyError
            gc_csr_free(c);
            gc_set_error("%lld", (long long)u);
            return GC_EKEY;
        }
        c->col[e] = pos;
    }
    c->flags = 0;
    *out = c;
    return GC_OK;
}

extern "C" int gc_json_write_coloring(const char* path, const int64_t* ids, const int32_t* colors, int64_t n) {
    if (!path || (n > 0 && !colors)) {
        gc_set_error("gc_json_write_coloring: null argument");
        return GC_EINVAL;
    }
    FILE* f = open_out(path);
    if (!f) return GC_EIO;
    Out o(f);
    if (n == 0) {
        o.puts_("[]");
    } else {
        o.puts_("[\n");
        for (int64_t i = 0; i < n; ++i) {
            o.puts_(i ? ",\n    {\n        \"id\": " : "    {\n        \"id\": ");
            o.num(ids ? ids[i] : i);
            o.puts_(",\n        \"color\": ");
            o.num(colors[i]);
            o.puts_("\n    }");
        }
        o.puts_("\n]");
    }
    return close_out(o, path);
}

extern "C" int gc_json_write_graph(const char* path, const int64_t* ids, const int64_t* row_ptr, const int32_t* col,
                                   int64_t n, const int32_t* colors) {
    if (!path || (n > 0 && (!row_ptr || (!col && row_ptr[n] > 0)))) {
        gc_set_error("gc_json_write_graph: null argument");
        return GC_EINVAL;
    }
    FILE* f = open_out(path);
    if (!f) return GC_EIO;
    Out o(f);
    if (n == 0) {
        o.puts_("[]");
    } else {
        o.puts_("[\n");
        for (int64_t i = 0; i < n; ++i) {
            o.puts_(i ? ",\n    {\n        \"id\": " : "    {\n        \"id\": ");
            o.num(ids ? ids[i] : i);
            o.puts_(",\n        \"neighbors\": ");
            const int64_t b = row_ptr[i], e = row_ptr[i + 1];
            if (b == e) {
                o.puts_("[]");
            } else {
                o.puts_("[\n");
                for (int64_t j = b; j < e; ++j) {
                    o.puts_(j > b ? ",\n            " : "            ");
                    o.num(ids ? ids[col[j]] : col[j]);
                }
                o.puts_("\n        ]");
            }
            o.puts_(",\n        \"color\": ");
            o.num(colors ? colors[i] : -1);
            o.puts_("\n    }");
        }
        o.puts_("\n]");
    }
    return close_out(o, path);
}

extern "C" int gc_csr_write(const char* path, const int64_t* row_ptr, const int32_t* col, const int64_t* ids, int64_t n,
                            int64_t nnz, uint32_t flags) {
    if (!path || n < 0 || nnz < 0 || !row_ptr || (nnz > 0 && !col)) {
        gc_set_error("gc_csr_write: bad argument");
        return GC_EINVAL;
    }
    FILE* f = open_out(path);
    if (!f) return GC_EIO;
    uint32_t has_ids = ids ? 1u : 0u;
    bool ok = fwrite(kMagic, 1, 8, f) == 8 && fwrite(&n, 8, 1, f) == 1 && fwrite(&nnz, 8, 1, f) == 1 &&
              fwrite(&flags, 4, 1, f) == 1 && fwrite(&has_ids, 4, 1, f) == 1 &&
              fwrite(row_ptr, 8, (size_t)(n + 1), f) == (size_t)(n + 1) &&
              (nnz == 0 || fwrite(col, 4, (size_t)nnz, f) == (size_t)nnz);
    if (ok && (nnz & 1)) {
        const int32_t pad = 0;
        ok = fwrite(&pad, 4, 1, f) == 1;
    }
    if (ok && ids && n > 0) ok = fwrite(ids, 8, (size_t)n, f) == (size_t)n;
    if (fclose(f) != 0) ok = false;
    if (!ok) {
        gc_set_error("write to %s failed: %s", path, strerror(errno));
        return GC_EIO;
    }
    return GC_OK;
}

extern "C" int gc_csr_read(const char* path, gc_csr** out) {
    if (!path || !out) {
        gc_set_error("gc_csr_read: null argument");
        return GC_EINVAL;
    }
    *out = nullptr;
    Mapped m;
    int rc = m.open_file(path);
    if (rc) return rc;
    if (m.len < 32 || memcmp(m.p, kMagic, 8) != 0) {
        gc_set_error("%s: not a GCSR file", path);
        return GC_EINVAL;
    }
    int64_t n, nnz;
    uint32_t flags, has_ids;
    memcpy(&n, m.p + 8, 8);
    memcpy(&nnz, m.p + 16, 8);
    memcpy(&flags, m.p + 24, 4);
    memcpy(&has_ids, m.p + 28, 4);
    // (nnz bounded by the file size first: 4 * nnz must not wrap the size arithmetic below)
    if (n < 0 || n > INT32_MAX || nnz < 0 || nnz > (int64_t)(m.len / 4) || has_ids > 1) {
        gc_set_error("%s: bad GCSR header (n=%lld nnz=%lld)", path, (long long)n, (long long)nnz);
        return GC_EINVAL;
    }
    const size_t off_col = 32 + 8 * (size_t)(n + 1);
    const size_t off_ids = off_col + 4 * (size_t)nnz + ((nnz & 1) ? 4 : 0);
    const size_t want = off_ids + (has_ids ? 8 * (size_t)n : 0);
    if (m.len != want) {
        gc_set_error("%s: GCSR size %zu, header implies %zu", path, m.len, want);
        return GC_EINVAL;
    }
    gc_csr* c = csr_new(n, nnz, has_ids != 0);
    if (!c) {
        gc_set_error("gc_csr_read: out of host memory");
        return GC_ENOMEM;
    }
    memcpy(c->row_ptr, m.p + 32, 8 * (size_t)(n + 1));
    if (nnz) memcpy(c->col, m.p + off_col, 4 * (size_t)nnz);
    if (has_ids && n) memcpy(c->ids, m.p + off_ids, 8 * (size_t)n);
    c->flags = flags;
    bool ok = c->row_ptr[0] == 0 && c->row_ptr[n] == nnz;
    for (int64_t i = 0; i < n && ok; ++i) ok = c->row_ptr[i] <= c->row_ptr[i + 1];
    for (int64_t e = 0; e < nnz && ok; ++e) ok = c->col[e] >= 0 && c->col[e] < n;
    if (!ok) {
        gc_csr_free(c);
        gc_set_error("%s: GCSR row_ptr / col out of range", path);
        return GC_EINVAL;
    }
    *out = c;
    return GC_OK;
}
