// Native reader and writer for the HDF5 subset of IGM's population files (.hss,
// actdist.hdf5); see include/igm_io.h for the scope.  Host C++ only: the population
// moves between the steps through this, in place of alabtools.HssFile / h5py
// (igm/core/step.py:346-396, igm/steps/ModelingStep.py:578-783,
// igm/steps/ActivationDistanceStep.py:234-298, igm/_preprocess.py:90-188).
//
// Format facts this file relies on (HDF5 File Format Specification, version 0
// superblock family -- what h5py writes with its default 'earliest' file format, as
// observed byte for byte in the reference's demo/demo_sample_outputs/*.hss files):
//   superblock 0: signature, 8 version/size bytes, group leaf/internal K (4, 16),
//     4 flag bytes, base / free-space / EOF / driver addresses, root symbol-table entry
//   symbol-table entry (40 B): name offset in the parent's local heap, object-header
//     address, cache type (1: scratch pad holds the group's B-tree and heap), scratch
//   group: B-tree v1 of type 0 (keys = local-heap offsets of names, children = SNOD
//     nodes of <= 2*leafK entries sorted by name) + local heap ("HEAP", names padded
//     to 8, offset 0 = "", free list 1 = none)
//   object header v1: version 1, message count, refcount, chunk size, 4 pad bytes,
//     then messages {type u16, size u16 (multiple of 8), flags u8, 3 reserved, data}
//   vlen data: {length u32, global-heap collection address u64, object index u32};
//     a collection ("GCOL", size >= 4096) holds objects {index u16, refcount u16,
//     4 reserved, size u64, data padded to 8}, index 0 = the free space
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "igm_io.h"

namespace {

thread_local std::string g_err;

int fail(const char* fmt, ...) {
    char b[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b, sizeof(b), fmt, ap);
    va_end(ap);
    g_err = b;
    return -1;
}

constexpr uint64_t kUndef = ~0ull;
const uint8_t kSig[8] = {0x89, 'H', 'D', 'F', '\r', '\n', 0x1a, '\n'};

struct Err {
    std::string msg;
};

[[noreturn]] void raise(const char* fmt, ...) {
    char b[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b, sizeof(b), fmt, ap);
    va_end(ap);
    throw Err{b};
}

uint64_t rd(const uint8_t* p, int n) {  // little-endian unsigned of n bytes
    uint64_t v = 0;
    for (int i = n - 1; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}

std::vector<std::string> split_path(const char* path) {
    std::vector<std::string> out;
    std::string cur;
    for (const char* c = path ? path : ""; *c; ++c) {
        if (*c == '/') {
            if (!cur.empty()) out.push_back(cur);
            cur.clear();
        } else {
            cur += *c;
        }
    }
    if (!cur.empty()) out.push_back(cur);
    return out;
}

// ============================================================== reader
struct Msg {
    int type;
    int flags;
    const uint8_t* p;
    size_t n;
};

struct Dtype {
    int cls = -1, size = 0, is_signed = 0;
};

struct Space {
    int rank = 0;
    int64_t dims[IGM_H5_MAXRANK] = {0};
    int64_t nelem = 1;
};

struct Filter {
    int id;
    int flags;
    std::vector<uint32_t> cd;
};

struct Layout {
    int cls = -1;  // 0 compact, 1 contiguous, 2 chunked
    uint64_t addr = kUndef, size = 0;
    const uint8_t* compact = nullptr;
    int ndim = 0;  // chunked: rank + 1
    uint32_t cdims[IGM_H5_MAXRANK + 1] = {0};
};

struct Attr {
    std::string name;
    Dtype t;
    Space s;
    const uint8_t* data;
    size_t n;
};

struct Object {
    std::vector<Msg> msgs;
    bool is_group = false;
    uint64_t btree = kUndef, heap = kUndef;
    Dtype t;
    Space s;
    Layout lay;
    std::vector<Filter> filters;
    std::vector<Attr> attrs;
};

}  // namespace

// the file's bytes: a read-only memory map (only the touched pages are read -- opening a
// population file to read its index does not read its coordinates)
struct FileBytes {
    const uint8_t* p = nullptr;
    size_t n = 0;
    ~FileBytes() {
        if (p) munmap(const_cast<uint8_t*>(p), n);
    }
    const uint8_t* data() const { return p; }
    size_t size() const { return n; }
};

struct igm_h5 {
    FileBytes buf;
    uint64_t base = 0, root = kUndef;
    int leafk = 4, intk = 16;
    std::map<std::string, uint64_t> paths;  // resolved object headers

    const uint8_t* at(uint64_t off, uint64_t n) const {
        if (off == kUndef || off + base < off || off + base + n > buf.size() || off + base + n < off)
            raise("HDF5: range [%llu, +%llu) outside the file (%zu bytes)", (unsigned long long)off,
                  (unsigned long long)n, buf.size());
        return buf.data() + base + off;
    }

    void parse_messages(const uint8_t* p, size_t n, size_t want, std::vector<Msg>& out,
                        std::vector<std::pair<uint64_t, uint64_t>>& cont) const {
        size_t o = 0;
        while (o + 8 <= n && out.size() < want) {
            const int type = (int)rd(p + o, 2), size = (int)rd(p + o + 2, 2), flags = p[o + 4];
            if (o + 8 + (size_t)size > n) raise("HDF5: object header message overruns its chunk");
            if (flags & 0x02) raise("HDF5: shared object-header messages are not supported");
            out.push_back(Msg{type, flags, p + o + 8, (size_t)size});
            if (type == 0x10) {
                if (size < 16) raise("HDF5: short continuation message");
                cont.emplace_back(rd(p + o + 8, 8), rd(p + o + 16, 8));
            }
            o += 8 + (size_t)size;
        }
    }

    std::vector<Msg> header(uint64_t addr) const {
        const uint8_t* h = at(addr, 16);
        if (h[0] != 1) {
            if (!memcmp(h, "OHDR", 4)) raise("HDF5: version-2 object headers (libver='latest') are not supported");
            raise("HDF5: object header version %d at %llu not supported", h[0], (unsigned long long)addr);
        }
        const size_t nmsg = rd(h + 2, 2), csize = rd(h + 8, 4);
        std::vector<Msg> out;
        std::vector<std::pair<uint64_t, uint64_t>> cont;
        parse_messages(at(addr + 16, csize), csize, nmsg, out, cont);
        for (size_t k = 0; k < cont.size() && out.size() < nmsg; ++k)
            parse_messages(at(cont[k].first, cont[k].second), cont[k].second, nmsg, out, cont);
        return out;
    }

    static Dtype dtype(const uint8_t* p, size_t n) {
        if (n < 8) raise("HDF5: short datatype message");
        Dtype t;
        t.cls = p[0] & 15;
        t.size = (int)rd(p + 4, 4);
        const uint8_t b0 = p[1];
        switch (t.cls) {
            case 0:
                if (b0 & 1) raise("HDF5: big-endian integers are not supported");
                t.is_signed = (b0 >> 3) & 1;
                if (t.size != 1 && t.size != 2 && t.size != 4 && t.size != 8) raise("HDF5: integer size %d", t.size);
                break;
            case 1:
                if (b0 & 1) raise("HDF5: big-endian floats are not supported");
                if (t.size != 4 && t.size != 8) raise("HDF5: float size %d", t.size);
                break;
            case 3:
                break;
            case 9:
                if ((b0 & 15) != 1) raise("HDF5: variable-length sequences (not strings) are not supported");
                break;
            default:
                raise("HDF5: datatype class %d is not supported", t.cls);
        }
        return t;
    }

    static Space space(const uint8_t* p, size_t n) {
        if (n < 4) raise("HDF5: short dataspace message");
        Space s;
        const int ver = p[0];
        s.rank = p[1];
        const int flags = p[2];
        if (s.rank > IGM_H5_MAXRANK) raise("HDF5: rank %d", s.rank);
        size_t o;
        if (ver == 1) {
            o = 8;
        } else if (ver == 2) {
            if (p[3] == 2) raise("HDF5: null dataspace");
            o = 4;
        } else {
            raise("HDF5: dataspace version %d", ver);
        }
        if (o + 8 * (size_t)s.rank * ((flags & 1) ? 2 : 1) > n) raise("HDF5: short dataspace message");
        s.nelem = 1;
        for (int d = 0; d < s.rank; ++d) {
            s.dims[d] = (int64_t)rd(p + o + 8 * d, 8);
            // a corrupt extent must not turn into a huge (or negative) allocation
            if (s.dims[d] < 0 || (s.dims[d] > 0 && s.nelem > ((int64_t)1 << 48) / s.dims[d]))
                raise("HDF5: implausible dataspace extent %lld in dimension %d", (long long)s.dims[d], d);
            s.nelem *= s.dims[d];
        }
        return s;
    }

    Object object(uint64_t addr) const {
        Object ob;
        ob.msgs = header(addr);
        bool have_t = false, have_s = false;
        for (const Msg& m : ob.msgs) {
            switch (m.type) {
                case 0x01:
                    ob.s = space(m.p, m.n);
                    have_s = true;
                    break;
                case 0x03:
                    ob.t = dtype(m.p, m.n);
                    have_t = true;
                    break;
                case 0x08: {
                    if (m.n < 2 || m.p[0] != 3) raise("HDF5: data layout version %d is not supported", m.n ? m.p[0] : -1);
                    ob.lay.cls = m.p[1];
                    // every field is checked against the message size before it is read
                    auto need = [&](size_t k) {
                        if (k > m.n) raise("HDF5: data layout message too short (%zu of %zu bytes)", (size_t)m.n, k);
                    };
                    if (ob.lay.cls == 0) {
                        need(4);
                        ob.lay.size = rd(m.p + 2, 2);
                        ob.lay.compact = m.p + 4;
                        if (4 + ob.lay.size > m.n) raise("HDF5: compact data overruns its message");
                    } else if (ob.lay.cls == 1) {
                        need(18);
                        ob.lay.addr = rd(m.p + 2, 8);
                        ob.lay.size = rd(m.p + 10, 8);
                    } else if (ob.lay.cls == 2) {
                        need(3);
                        ob.lay.ndim = m.p[2];
                        if (ob.lay.ndim < 1 || ob.lay.ndim > IGM_H5_MAXRANK + 1) raise("HDF5: chunk rank");
                        need(11 + 4 * (size_t)ob.lay.ndim);
                        ob.lay.addr = rd(m.p + 3, 8);
                        for (int d = 0; d < ob.lay.ndim; ++d) ob.lay.cdims[d] = (uint32_t)rd(m.p + 11 + 4 * d, 4);
                    } else {
                        raise("HDF5: layout class %d", ob.lay.cls);
                    }
                    break;
                }
                case 0x0B: {
                    auto need = [&](size_t k) {
                        if (k > m.n) raise("HDF5: filter pipeline message too short (%zu of %zu bytes)", (size_t)m.n, k);
                    };
                    need(2);
                    const int ver = m.p[0], nf = m.p[1];
                    size_t o = ver == 1 ? 8 : 2;
                    need(o);
                    for (int k = 0; k < nf; ++k) {
                        Filter f;
                        need(o + 2);
                        f.id = (int)rd(m.p + o, 2);
                        size_t namelen = 0;
                        if (ver == 1 || f.id >= 256) {
                            need(o + 4);
                            namelen = rd(m.p + o + 2, 2);
                            o += 2;
                        }
                        need(o + 6);
                        f.flags = (int)rd(m.p + o + 2, 2);
                        const int ncd = (int)rd(m.p + o + 4, 2);
                        o += 6;
                        if (ver == 1) namelen = (namelen + 7) & ~size_t(7);
                        o += namelen;
                        need(o + 4 * (size_t)ncd);
                        for (int c = 0; c < ncd; ++c) f.cd.push_back((uint32_t)rd(m.p + o + 4 * c, 4));
                        o += 4 * (size_t)ncd;
                        if (ver == 1 && (ncd & 1)) o += 4;
                        if (o > m.n) raise("HDF5: filter pipeline overruns its message");
                        ob.filters.push_back(f);
                    }
                    break;
                }
                case 0x0C: {
                    Attr a;
                    const int ver = m.p[0];
                    const size_t nl = rd(m.p + 2, 2), tl = rd(m.p + 4, 2), sl = rd(m.p + 6, 2);
                    size_t o = ver == 3 ? 9 : 8;
                    auto pad = [&](size_t x) { return ver == 1 ? ((x + 7) & ~size_t(7)) : x; };
                    if (ver < 1 || ver > 3) raise("HDF5: attribute message version %d", ver);
                    if (ver >= 2 && (m.p[1] & 3)) raise("HDF5: shared attribute datatypes are not supported");
                    if (o + pad(nl) + pad(tl) + pad(sl) > m.n) raise("HDF5: attribute overruns its message");
                    a.name.assign((const char*)m.p + o, nl ? strnlen((const char*)m.p + o, nl) : 0);
                    o += pad(nl);
                    a.t = dtype(m.p + o, tl);
                    o += pad(tl);
                    a.s = space(m.p + o, sl);
                    o += pad(sl);
                    a.data = m.p + o;
                    a.n = m.n - o;
                    if ((size_t)a.s.nelem * a.t.size > a.n) raise("HDF5: attribute '%s' data overruns", a.name.c_str());
                    ob.attrs.push_back(a);
                    break;
                }
                case 0x11:
                    ob.is_group = true;
                    ob.btree = rd(m.p, 8);
                    ob.heap = rd(m.p + 8, 8);
                    break;
                case 0x02:
                case 0x06:
                    raise("HDF5: link-message (new style) groups are not supported");
                case 0x15:
                    raise("HDF5: dense attribute storage is not supported");
                default:
                    break;
            }
        }
        if (!ob.is_group && (!have_t || !have_s || ob.lay.cls < 0)) raise("HDF5: object is neither a group nor a dataset");
        return ob;
    }

    // (name, object header) of every member of a group, in B-tree order
    void members(uint64_t btree, uint64_t heap, std::vector<std::pair<std::string, uint64_t>>& out) const {
        const uint8_t* h = at(heap, 32);
        if (memcmp(h, "HEAP", 4)) raise("HDF5: bad local heap signature");
        const uint64_t dsize = rd(h + 8, 8), daddr = rd(h + 24, 8);
        const uint8_t* names = at(daddr, dsize);
        const uint8_t* b = at(btree, 24);
        if (memcmp(b, "TREE", 4) || b[4] != 0) raise("HDF5: bad group B-tree node");
        const int level = b[5], n = (int)rd(b + 6, 2);
        const uint8_t* kc = at(btree + 24, (size_t)(2 * n + 1) * 8);
        for (int i = 0; i < n; ++i) {
            const uint64_t child = rd(kc + 8 + 16 * (size_t)i, 8);
            if (level > 0) {
                members(child, heap, out);
                continue;
            }
            const uint8_t* s = at(child, 8);
            if (memcmp(s, "SNOD", 4)) raise("HDF5: bad symbol-table node signature");
            const int ns = (int)rd(s + 6, 2);
            const uint8_t* e = at(child + 8, (size_t)ns * 40);
            for (int k = 0; k < ns; ++k) {
                const uint64_t off = rd(e + 40 * k, 8);
                if (off >= dsize) raise("HDF5: symbol name offset outside its heap");
                out.emplace_back(std::string((const char*)names + off, strnlen((const char*)names + off, dsize - off)),
                                 rd(e + 40 * k + 8, 8));
            }
        }
    }

    uint64_t resolve(const char* path) {
        auto it = paths.find(path ? path : "");
        if (it != paths.end()) return it->second;
        uint64_t cur = root;
        for (const std::string& c : split_path(path)) {
            const Object ob = object(cur);
            if (!ob.is_group) raise("HDF5: '%s' is not a group on the way to '%s'", c.c_str(), path);
            std::vector<std::pair<std::string, uint64_t>> ms;
            members(ob.btree, ob.heap, ms);
            uint64_t nxt = kUndef;
            for (auto& m : ms)
                if (m.first == c) nxt = m.second;
            if (nxt == kUndef) raise("HDF5: no object '%s' (in '%s')", c.c_str(), path);
            cur = nxt;
        }
        paths[path ? path : ""] = cur;
        return cur;
    }

    // global-heap object (collection address, index)
    std::string gheap(uint64_t coll, uint32_t index) const {
        const uint8_t* h = at(coll, 16);
        if (memcmp(h, "GCOL", 4)) raise("HDF5: bad global heap signature");
        const uint64_t csize = rd(h + 8, 8);
        const uint8_t* c = at(coll, csize);
        uint64_t o = 16;
        while (o + 16 <= csize) {
            const uint32_t idx = (uint32_t)rd(c + o, 2);
            const uint64_t sz = rd(c + o + 8, 8);
            if (idx == 0) break;  // free space
            if (o + 16 + sz > csize) raise("HDF5: global heap object overruns its collection");
            if (idx == index) return std::string((const char*)c + o + 16, sz);
            o += 16 + ((sz + 7) & ~uint64_t(7));
        }
        raise("HDF5: global heap object %u not found", index);
    }

    void unfilter(std::vector<uint8_t>& data, size_t raw, const std::vector<Filter>& fl, uint32_t mask,
                  int elsize) const {
        for (int k = (int)fl.size() - 1; k >= 0; --k) {
            if (mask & (1u << k)) continue;
            const Filter& f = fl[k];
            if (f.id == 1) {  // deflate
                std::vector<uint8_t> out(raw);
                uLongf n = (uLongf)raw;
                const int rc = uncompress(out.data(), &n, data.data(), (uLong)data.size());
                if (rc != Z_OK || n != raw) raise("HDF5: deflate failed (zlib %d, %lu of %zu bytes)", rc, (unsigned long)n, raw);
                data.swap(out);
            } else if (f.id == 2) {  // shuffle
                const size_t es = f.cd.empty() ? (size_t)elsize : f.cd[0];
                if (es > 1 && data.size() >= es) {
                    const size_t ne = data.size() / es;
                    std::vector<uint8_t> out(data);
                    for (size_t b = 0; b < es; ++b)
                        for (size_t e = 0; e < ne; ++e) out[e * es + b] = data[b * ne + e];
                    data.swap(out);
                }
            } else if (f.id == 3) {  // fletcher32: the checksum trails the data
                if (data.size() < 4) raise("HDF5: fletcher32 chunk too short");
                data.resize(data.size() - 4);
            } else {
                raise("HDF5: filter %d is not supported", f.id);
            }
        }
    }

    void read_chunks(uint64_t node, const Object& ob, uint8_t* out) const {
        const int D = ob.lay.ndim, r = D - 1, es = ob.t.size;
        const size_t ksz = 8 + 8 * (size_t)D;
        const uint8_t* b = at(node, 24);
        if (memcmp(b, "TREE", 4) || b[4] != 1) raise("HDF5: bad chunk B-tree node");
        const int level = b[5], n = (int)rd(b + 6, 2);
        const uint8_t* kc = at(node + 24, (size_t)n * (ksz + 8) + ksz);
        size_t craw = es;
        for (int d = 0; d < r; ++d) craw *= ob.lay.cdims[d];
        for (int i = 0; i < n; ++i) {
            const uint8_t* key = kc + (size_t)i * (ksz + 8);
            const uint64_t child = rd(key + ksz, 8);
            if (level > 0) {
                read_chunks(child, ob, out);
                continue;
            }
            const uint32_t nbytes = (uint32_t)rd(key, 4), mask = (uint32_t)rd(key + 4, 4);
            int64_t off[IGM_H5_MAXRANK];
            for (int d = 0; d < r; ++d) {
                off[d] = (int64_t)rd(key + 8 + 8 * d, 8);
                // a chunk must start inside the dataset (the copy below writes from there)
                if (off[d] < 0 || off[d] >= ob.s.dims[d] || (ob.lay.cdims[d] && off[d] % ob.lay.cdims[d]))
                    raise("HDF5: chunk offset %lld outside dimension %d (extent %lld)", (long long)off[d], d,
                          (long long)ob.s.dims[d]);
            }
            const uint8_t* src = at(child, nbytes);
            std::vector<uint8_t> data(src, src + nbytes);
            unfilter(data, craw, ob.filters, mask, es);
            if (data.size() != craw) raise("HDF5: chunk of %zu bytes, expected %zu", data.size(), craw);
            // copy the chunk's part inside the dataset extent, a last-dimension run at a time
            int64_t idx[IGM_H5_MAXRANK] = {0};
            const int64_t cl = ob.lay.cdims[r - 1];
            const int64_t run = std::min<int64_t>(cl, ob.s.dims[r - 1] - off[r - 1]);
            if (run <= 0) continue;
            for (;;) {
                bool inside = true;
                int64_t g = 0, c = 0;
                for (int d = 0; d < r; ++d) {
                    const int64_t gd = off[d] + idx[d];
                    if (gd >= ob.s.dims[d]) inside = false;
                    g = g * ob.s.dims[d] + gd;
                    c = c * ob.lay.cdims[d] + idx[d];
                }
                if (inside) memcpy(out + g * es, data.data() + c * es, (size_t)run * es);
                int d = r - 2;
                for (; d >= 0; --d) {
                    if (++idx[d] < (int64_t)ob.lay.cdims[d]) break;
                    idx[d] = 0;
                }
                if (d < 0) break;
            }
        }
    }

    void read_data(const Object& ob, uint8_t* out, size_t nbytes) const {
        if (ob.lay.cls == 0) {
            if (ob.lay.size < nbytes) raise("HDF5: compact data smaller than the dataset");
            memcpy(out, ob.lay.compact, nbytes);
        } else if (ob.lay.cls == 1) {
            if (ob.lay.addr == kUndef) {
                memset(out, 0, nbytes);  // never written: the fill value (0)
                return;
            }
            if (!ob.filters.empty()) raise("HDF5: filtered contiguous data");
            memcpy(out, at(ob.lay.addr, nbytes), nbytes);
        } else {
            if (ob.lay.ndim != ob.s.rank + 1 || (int)ob.lay.cdims[ob.s.rank] != ob.t.size)
                raise("HDF5: chunk dimensions do not match the dataspace");
            memset(out, 0, nbytes);
            if (ob.lay.addr != kUndef && nbytes) read_chunks(ob.lay.addr, ob, out);
        }
    }

    struct Target {
        Object ob;
        const Attr* a = nullptr;
    };

    // the dataset's raw bytes or the attribute's data
    void bytes(Target& tg, std::vector<uint8_t>& v) const {
        const Dtype& t = tg.a ? tg.a->t : tg.ob.t;
        const Space& s = tg.a ? tg.a->s : tg.ob.s;
        v.resize((size_t)s.nelem * t.size);
        if (tg.a)
            memcpy(v.data(), tg.a->data, v.size());
        else
            read_data(tg.ob, v.data(), v.size());
    }
};

namespace {

void target(igm_h5* f, const char* path, const char* attr, igm_h5::Target& tg) {
    tg.ob = f->object(f->resolve(path));
    tg.a = nullptr;
    if (attr) {
        for (const Attr& a : tg.ob.attrs)
            if (a.name == attr) tg.a = &a;
        if (!tg.a) raise("HDF5: '%s' has no attribute '%s'", path, attr);
    } else if (tg.ob.is_group) {
        raise("HDF5: '%s' is a group, not a dataset", path);
    }
}

int copy_names(const std::string& s, char* names, size_t cap, size_t* needed) {
    if (needed) *needed = s.size() + 1;
    if (names && cap) {
        const size_t n = std::min(cap - 1, s.size());
        memcpy(names, s.data(), n);
        names[n] = 0;
    }
    return 0;
}

}  // namespace

extern "C" const char* igm_io_last_error(void) { return g_err.c_str(); }

extern "C" int igm_h5_open(const char* path, igm_h5** out) {
    if (!path || !out) return fail("igm_h5_open: null argument");
    *out = nullptr;
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return fail("igm_h5_open: cannot open '%s'", path);
    std::unique_ptr<igm_h5> f(new igm_h5());
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        return fail("igm_h5_open: cannot stat '%s'", path);
    }
    if (st.st_size > 0) {
        void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) {
            close(fd);
            return fail("igm_h5_open: cannot map '%s'", path);
        }
        f->buf.p = static_cast<const uint8_t*>(m);
        f->buf.n = (size_t)st.st_size;
    }
    close(fd);
    try {
        // the superblock may sit at 0, 512, 1024, ... (a user block before it)
        size_t sb = kUndef;
        for (size_t o = 0; o + 8 <= f->buf.size(); o = o ? 2 * o : 512)
            if (!memcmp(f->buf.data() + o, kSig, 8)) {
                sb = o;
                break;
            }
        if (sb == kUndef) return fail("igm_h5_open: '%s' is not an HDF5 file", path);
        const uint8_t* p = f->buf.data() + sb;
        if (f->buf.size() < sb + 96) return fail("igm_h5_open: truncated superblock");
        const int ver = p[8];
        if (ver > 1) return fail("igm_h5_open: superblock version %d (libver='latest') is not supported", ver);
        if (p[13] != 8 || p[14] != 8) return fail("igm_h5_open: offset/length sizes %d/%d not supported", p[13], p[14]);
        f->leafk = (int)rd(p + 16, 2);
        f->intk = (int)rd(p + 18, 2);
        const size_t a = ver == 1 ? 28 : 24;
        f->base = rd(p + a, 8) == kUndef ? sb : rd(p + a, 8);
        f->root = rd(p + a + 32 + 8, 8);  // root symbol-table entry: name offset, header address
        f->paths[""] = f->root;
        f->object(f->root);  // the root must parse
    } catch (const Err& e) {
        return fail("%s ('%s')", e.msg.c_str(), path);
    }
    *out = f.release();
    return 0;
}

extern "C" int igm_h5_close(igm_h5* f) {
    delete f;
    return 0;
}

extern "C" int igm_h5_list(igm_h5* f, const char* group, char* names, size_t cap, size_t* needed) {
    if (!f) return fail("igm_h5_list: null file");
    try {
        const Object ob = f->object(f->resolve(group));
        if (!ob.is_group) return fail("igm_h5_list: '%s' is not a group", group ? group : "/");
        std::vector<std::pair<std::string, uint64_t>> ms;
        f->members(ob.btree, ob.heap, ms);
        std::string s;
        for (auto& m : ms) {
            if (!s.empty()) s += '\n';
            s += m.first;
            if (f->object(m.second).is_group) s += '/';
        }
        return copy_names(s, names, cap, needed);
    } catch (const Err& e) {
        return fail("%s", e.msg.c_str());
    }
}

extern "C" int igm_h5_attr_names(igm_h5* f, const char* path, char* names, size_t cap, size_t* needed) {
    if (!f) return fail("igm_h5_attr_names: null file");
    try {
        const Object ob = f->object(f->resolve(path));
        std::string s;
        for (const Attr& a : ob.attrs) {
            if (!s.empty()) s += '\n';
            s += a.name;
        }
        return copy_names(s, names, cap, needed);
    } catch (const Err& e) {
        return fail("%s", e.msg.c_str());
    }
}

extern "C" int igm_h5_info_of(igm_h5* f, const char* path, const char* attr, igm_h5_info* info) {
    if (!f || !info) return fail("igm_h5_info_of: null argument");
    try {
        igm_h5::Target tg;
        target(f, path, attr, tg);
        const Dtype& t = tg.a ? tg.a->t : tg.ob.t;
        const Space& s = tg.a ? tg.a->s : tg.ob.s;
        memset(info, 0, sizeof(*info));
        info->cls = t.cls;
        info->size = t.size;
        info->is_signed = t.is_signed;
        info->rank = s.rank;
        for (int d = 0; d < s.rank; ++d) info->dims[d] = s.dims[d];
        info->nelem = s.nelem;
        // contiguous raw data must lie inside the file (checked here, before a caller
        // allocates the dataset's size)
        if (!tg.a && tg.ob.lay.cls == 1 && tg.ob.lay.addr != kUndef && tg.ob.filters.empty())
            (void)f->at(tg.ob.lay.addr, (uint64_t)s.nelem * (uint64_t)t.size);
        info->layout = tg.a ? -1 : tg.ob.lay.cls;
        info->nfilter = tg.a ? 0 : (int)tg.ob.filters.size();
        info->data_offset = (!tg.a && tg.ob.lay.cls == 1 && tg.ob.lay.addr != kUndef && tg.ob.filters.empty())
                                ? (int64_t)(tg.ob.lay.addr + f->base)
                                : -1;
        return 0;
    } catch (const Err& e) {
        return fail("%s", e.msg.c_str());
    }
}

extern "C" int igm_h5_read(igm_h5* f, const char* path, const char* attr, void* out, size_t nbytes) {
    if (!f || (!out && nbytes)) return fail("igm_h5_read: null argument");
    try {
        igm_h5::Target tg;
        target(f, path, attr, tg);
        const Dtype& t = tg.a ? tg.a->t : tg.ob.t;
        const Space& s = tg.a ? tg.a->s : tg.ob.s;
        if (t.cls == IGM_H5_VLSTR) return fail("igm_h5_read: '%s' holds variable-length strings", path);
        if ((size_t)s.nelem * t.size != nbytes)
            return fail("igm_h5_read: '%s' has %lld x %d bytes, buffer %zu", path, (long long)s.nelem, t.size, nbytes);
        if (tg.a)
            memcpy(out, tg.a->data, nbytes);
        else
            f->read_data(tg.ob, (uint8_t*)out, nbytes);
        return 0;
    } catch (const Err& e) {
        return fail("%s", e.msg.c_str());
    }
}

extern "C" int igm_h5_read_vlstr(igm_h5* f, const char* path, const char* attr, int64_t index, char* out, size_t cap,
                                 size_t* len) {
    if (!f) return fail("igm_h5_read_vlstr: null file");
    try {
        igm_h5::Target tg;
        target(f, path, attr, tg);
        const Dtype& t = tg.a ? tg.a->t : tg.ob.t;
        const Space& s = tg.a ? tg.a->s : tg.ob.s;
        if (t.cls != IGM_H5_VLSTR) return fail("igm_h5_read_vlstr: '%s' is not a vlen string", path);
        if (index < 0 || index >= s.nelem) return fail("igm_h5_read_vlstr: index %lld out of range", (long long)index);
        std::vector<uint8_t> v;
        f->bytes(tg, v);
        const uint8_t* e = v.data() + 16 * index;
        const uint32_t n = (uint32_t)rd(e, 4);
        const uint64_t coll = rd(e + 4, 8);
        const uint32_t id = (uint32_t)rd(e + 12, 4);
        std::string str = n ? f->gheap(coll, id) : std::string();
        if (str.size() > n) str.resize(n);
        if (len) *len = str.size();
        if (out && cap) memcpy(out, str.data(), std::min(cap, str.size()));
        return 0;
    } catch (const Err& e) {
        return fail("%s", e.msg.c_str());
    }
}

// ============================================================== writer
namespace {

struct WAttr {
    std::string name;
    std::vector<uint8_t> dt, ds, data;
    bool vl = false;
    std::string vstr;
};

struct WNode {
    std::string name;
    bool group = true;
    std::vector<std::unique_ptr<WNode>> kids;
    std::vector<WAttr> attrs;
    // dataset
    std::vector<uint8_t> dt, ds, data;
    bool vl = false;
    std::string vstr;
    // layout pass
    uint64_t ohdr = 0, btree = 0, heap = 0, heapdata = 0, raw = kUndef;
    std::vector<uint64_t> snods;
    std::vector<uint64_t> name_off;  // per sorted kid: its name's offset in this group's heap
    std::vector<uint8_t> heapbytes;
    uint32_t vid = 0;  // global heap index of a vlen string dataset
    std::vector<uint32_t> attr_vid;
    size_t hdr_size = 0;
};

void put(std::vector<uint8_t>& b, uint64_t v, int n) {
    for (int i = 0; i < n; ++i) b.push_back((uint8_t)(v >> (8 * i)));
}
void pad8(std::vector<uint8_t>& b) {
    while (b.size() & 7) b.push_back(0);
}

std::vector<uint8_t> dtype_bytes(int cls, int size, int is_signed) {
    std::vector<uint8_t> b;
    if (cls == IGM_H5_INT) {
        if (size != 1 && size != 2 && size != 4 && size != 8) raise("integer size %d", size);
        b = {0x10, (uint8_t)(is_signed ? 0x08 : 0x00), 0, 0};
        put(b, size, 4);
        put(b, 0, 2);
        put(b, 8 * size, 2);
    } else if (cls == IGM_H5_FLOAT) {
        if (size != 4 && size != 8) raise("float size %d", size);
        const bool d = size == 8;
        b = {0x11, 0x20, (uint8_t)(d ? 63 : 31), 0};
        put(b, size, 4);
        put(b, 0, 2);
        put(b, 8 * size, 2);
        b.push_back(d ? 52 : 23);  // exponent location
        b.push_back(d ? 11 : 8);   // exponent size
        b.push_back(0);            // mantissa location
        b.push_back(d ? 52 : 23);  // mantissa size
        put(b, d ? 1023 : 127, 4);
    } else if (cls == IGM_H5_STRING) {
        if (size < 1) raise("string size %d", size);
        b = {0x13, 0x01, 0, 0};  // null-padded ASCII (numpy 'S<n>')
        put(b, size, 4);
    } else if (cls == IGM_H5_VLSTR) {
        b = {0x19, 0x01, 0x01, 0};  // vlen string, null-terminated, UTF-8 (h5py str)
        put(b, 16, 4);
        const uint8_t base[12] = {0x10, 0, 0, 0, 1, 0, 0, 0, 0, 0, 8, 0};  // unsigned char
        b.insert(b.end(), base, base + 12);
    } else {
        raise("datatype class %d not writable", cls);
    }
    return b;
}

std::vector<uint8_t> space_bytes(int rank, const int64_t* dims) {
    if (rank < 0 || rank > IGM_H5_MAXRANK) raise("rank %d", rank);
    std::vector<uint8_t> b = {1, (uint8_t)rank, (uint8_t)(rank ? 1 : 0), 0, 0, 0, 0, 0};
    for (int r = 0; r < 2 && rank; ++r)  // dimensions, then the (equal) maximum dimensions
        for (int d = 0; d < rank; ++d) {
            if (dims[d] < 0) raise("negative dimension");
            put(b, (uint64_t)dims[d], 8);
        }
    return b;
}

}  // namespace

struct igm_h5w {
    std::string path;
    WNode root;
    std::vector<std::string> vl;  // global heap objects, index = position + 1

    WNode* node(const std::vector<std::string>& parts, size_t n, bool create) {
        WNode* cur = &root;
        for (size_t i = 0; i < n; ++i) {
            WNode* nxt = nullptr;
            for (auto& k : cur->kids)
                if (k->name == parts[i]) nxt = k.get();
            if (!nxt) {
                if (!create) raise("no object '%s'", parts[i].c_str());
                cur->kids.emplace_back(new WNode());
                nxt = cur->kids.back().get();
                nxt->name = parts[i];
            }
            if (!nxt->group && i + 1 < n) raise("'%s' is a dataset, not a group", parts[i].c_str());
            cur = nxt;
        }
        return cur;
    }

    WNode* new_leaf(const char* path) {
        const auto parts = split_path(path);
        if (parts.empty()) raise("empty dataset path");
        WNode* parent = node(parts, parts.size() - 1, true);
        if (!parent->group) raise("parent of '%s' is a dataset", path);
        for (auto& k : parent->kids)
            if (k->name == parts.back()) raise("'%s' already exists", path);
        parent->kids.emplace_back(new WNode());
        WNode* d = parent->kids.back().get();
        d->name = parts.back();
        d->group = false;
        return d;
    }

    // ---- layout
    std::vector<uint8_t> out;
    uint64_t gcol = kUndef, gcol_size = 0;

    static size_t msg_size(size_t data) { return 8 + ((data + 7) & ~size_t(7)); }

    static std::vector<uint8_t> attr_msg(const WAttr& a, uint64_t gcol, uint32_t vid) {
        std::vector<uint8_t> m = {1, 0};
        put(m, a.name.size() + 1, 2);
        put(m, a.dt.size(), 2);
        put(m, a.ds.size(), 2);
        m.insert(m.end(), a.name.begin(), a.name.end());
        m.push_back(0);
        pad8(m);
        m.insert(m.end(), a.dt.begin(), a.dt.end());
        pad8(m);
        m.insert(m.end(), a.ds.begin(), a.ds.end());
        pad8(m);
        if (a.vl) {
            put(m, a.vstr.size(), 4);
            put(m, gcol, 8);
            put(m, vid, 4);
        } else {
            m.insert(m.end(), a.data.begin(), a.data.end());
        }
        return m;
    }

    // the messages of an object header (data only; flags per message)
    std::vector<std::pair<std::pair<int, int>, std::vector<uint8_t>>> messages(const WNode& n) const {
        std::vector<std::pair<std::pair<int, int>, std::vector<uint8_t>>> ms;
        if (n.group) {
            std::vector<uint8_t> st;
            put(st, n.btree, 8);
            put(st, n.heap, 8);
            ms.push_back({{0x11, 0}, st});
        } else {
            ms.push_back({{0x01, 0}, n.ds});
            ms.push_back({{0x03, 1}, n.dt});
            ms.push_back({{0x05, 1}, {2, 2, 0, 1, 0, 0, 0, 0}});  // fill value v2: late alloc, defined, size 0
            std::vector<uint8_t> lay = {3, 1};
            const uint64_t nbytes = n.vl ? 16 : n.data.size();
            put(lay, nbytes ? n.raw : kUndef, 8);
            put(lay, nbytes, 8);
            ms.push_back({{0x08, 0}, lay});
        }
        for (size_t i = 0; i < n.attrs.size(); ++i)
            ms.push_back({{0x0C, 0}, attr_msg(n.attrs[i], gcol, n.attr_vid.empty() ? 0 : n.attr_vid[i])});
        return ms;
    }

    size_t header_bytes(const WNode& n) const {
        size_t s = 0;
        for (auto& m : messages(n)) s += msg_size(m.second.size());
        return 16 + std::max<size_t>(s, 256 - 16);
    }

    static std::vector<WNode*> sorted_kids(WNode& n) {
        std::vector<WNode*> v;
        for (auto& k : n.kids) v.push_back(k.get());
        std::sort(v.begin(), v.end(), [](WNode* a, WNode* b) { return strcmp(a->name.c_str(), b->name.c_str()) < 0; });
        return v;
    }

    static constexpr int kLeafK = 4, kIntK = 16;
    static constexpr size_t kBtreeBytes = 24 + (2 * kIntK) * 8 + (2 * kIntK + 1) * 8;
    static constexpr size_t kSnodBytes = 8 + 2 * kLeafK * 40;

    void assign_vl(WNode& n) {
        if (!n.group && n.vl) {
            vl.push_back(n.vstr);
            n.vid = (uint32_t)vl.size();
        }
        n.attr_vid.assign(n.attrs.size(), 0);
        for (size_t i = 0; i < n.attrs.size(); ++i)
            if (n.attrs[i].vl) {
                vl.push_back(n.attrs[i].vstr);
                n.attr_vid[i] = (uint32_t)vl.size();
            }
        for (auto& k : n.kids) assign_vl(*k);
    }

    // metadata addresses, depth first
    void place_meta(WNode& n, uint64_t& at) {
        n.ohdr = at;
        at += header_bytes(n);
        if (!n.group) return;
        auto kids = sorted_kids(n);
        const size_t nsnod = (kids.size() + 2 * kLeafK - 1) / (2 * kLeafK);  // an empty group: no node
        if (nsnod > 2 * kIntK) raise("group '%s' has more than %d members", n.name.c_str(), 2 * kIntK * 2 * kLeafK);
        n.btree = at;
        at += kBtreeBytes;
        n.snods.clear();
        for (size_t s = 0; s < nsnod; ++s) {
            n.snods.push_back(at);
            at += kSnodBytes;
        }
        // local heap: "" at 0, then the names padded to 8
        n.heapbytes.assign(8, 0);
        n.name_off.clear();
        for (WNode* k : kids) {
            n.name_off.push_back(n.heapbytes.size());
            n.heapbytes.insert(n.heapbytes.end(), k->name.begin(), k->name.end());
            n.heapbytes.push_back(0);
            pad8(n.heapbytes);
        }
        n.heap = at;
        n.heapdata = at + 32;
        at += 32 + n.heapbytes.size();
        for (WNode* k : kids) place_meta(*k, at);
    }

    void place_raw(WNode& n, uint64_t& at) {
        if (!n.group) {
            const uint64_t nb = n.vl ? 16 : n.data.size();
            n.raw = nb ? at : kUndef;
            at += (nb + 7) & ~uint64_t(7);
        }
        for (WNode* k : sorted_kids(n)) place_raw(*k, at);
    }

    void emit_at(uint64_t addr, const std::vector<uint8_t>& b) {
        if (addr + b.size() > out.size()) raise("internal: write past the laid-out file");
        memcpy(out.data() + addr, b.data(), b.size());
    }

    void emit_header(const WNode& n) {
        auto ms = messages(n);
        std::vector<uint8_t> body;
        for (auto& m : ms) {
            put(body, m.first.first, 2);
            put(body, (m.second.size() + 7) & ~size_t(7), 2);
            body.push_back((uint8_t)m.first.second);
            body.insert(body.end(), 3, 0);
            body.insert(body.end(), m.second.begin(), m.second.end());
            pad8(body);
        }
        size_t nmsg = ms.size();
        const size_t csize = header_bytes(n) - 16;
        if (body.size() < csize) {  // a NIL message fills the rest of the chunk
            const size_t rest = csize - body.size() - 8;
            put(body, 0, 2);
            put(body, rest, 2);
            body.insert(body.end(), 4 + rest, 0);
            ++nmsg;
        }
        std::vector<uint8_t> h = {1, 0};
        put(h, nmsg, 2);
        put(h, 1, 4);
        put(h, csize, 4);
        put(h, 0, 4);
        h.insert(h.end(), body.begin(), body.end());
        emit_at(n.ohdr, h);
    }

    void emit(WNode& n) {
        emit_header(n);
        if (!n.group) {
            if (n.vl) {
                std::vector<uint8_t> e;
                put(e, n.vstr.size(), 4);
                put(e, gcol, 8);
                put(e, n.vid, 4);
                emit_at(n.raw, e);
            } else if (!n.data.empty()) {
                emit_at(n.raw, n.data);
            }
            return;
        }
        auto kids = sorted_kids(n);
        const size_t nsnod = n.snods.size();
        // B-tree (type 0, one leaf level): key 0 = "", key i+1 = last name of SNOD i
        std::vector<uint8_t> bt = {'T', 'R', 'E', 'E', 0, 0};
        put(bt, nsnod, 2);
        put(bt, kUndef, 8);
        put(bt, kUndef, 8);
        put(bt, 0, 8);
        for (size_t s = 0; s < nsnod; ++s) {
            put(bt, n.snods[s], 8);
            const size_t last = std::min(kids.size(), (s + 1) * 2 * kLeafK);
            put(bt, last ? n.name_off[last - 1] : 0, 8);
        }
        bt.resize(kBtreeBytes, 0);
        emit_at(n.btree, bt);
        for (size_t s = 0; s < nsnod; ++s) {
            const size_t k0 = s * 2 * kLeafK, k1 = std::min(kids.size(), k0 + 2 * kLeafK);
            std::vector<uint8_t> sn = {'S', 'N', 'O', 'D', 1, 0};
            put(sn, k1 - k0, 2);
            for (size_t k = k0; k < k1; ++k) {
                put(sn, n.name_off[k], 8);
                put(sn, kids[k]->ohdr, 8);
                if (kids[k]->group) {  // cache type 1: the group's B-tree and heap
                    put(sn, 1, 4);
                    put(sn, 0, 4);
                    put(sn, kids[k]->btree, 8);
                    put(sn, kids[k]->heap, 8);
                } else {
                    sn.insert(sn.end(), 24, 0);
                }
            }
            sn.resize(kSnodBytes, 0);
            emit_at(n.snods[s], sn);
        }
        std::vector<uint8_t> hp = {'H', 'E', 'A', 'P', 0, 0, 0, 0};
        put(hp, n.heapbytes.size(), 8);
        put(hp, 1, 8);  // no free block
        put(hp, n.heapdata, 8);
        hp.insert(hp.end(), n.heapbytes.begin(), n.heapbytes.end());
        emit_at(n.heap, hp);
        for (WNode* k : kids) emit(*k);
    }

    void write() {
        assign_vl(root);
        uint64_t at = 96;
        place_meta(root, at);
        if (!vl.empty()) {  // one global heap collection (>= 4096 bytes, free space last)
            gcol = at;
            uint64_t sz = 16;
            for (auto& s : vl) sz += 16 + ((s.size() + 7) & ~size_t(7));
            gcol_size = std::max<uint64_t>(sz + 16, 4096);
            at += gcol_size;
        }
        place_raw(root, at);
        out.assign(at, 0);
        // superblock 0
        std::vector<uint8_t> sb(kSig, kSig + 8);
        const uint8_t vers[8] = {0, 0, 0, 0, 0, 8, 8, 0};
        sb.insert(sb.end(), vers, vers + 8);
        put(sb, kLeafK, 2);
        put(sb, kIntK, 2);
        put(sb, 0, 4);
        put(sb, 0, 8);       // base address
        put(sb, kUndef, 8);  // free-space info
        put(sb, at, 8);      // end of file
        put(sb, kUndef, 8);  // driver info
        put(sb, 0, 8);       // root entry: name offset
        put(sb, root.ohdr, 8);
        put(sb, 1, 4);
        put(sb, 0, 4);
        put(sb, root.btree, 8);
        put(sb, root.heap, 8);
        emit_at(0, sb);
        if (!vl.empty()) {
            std::vector<uint8_t> g = {'G', 'C', 'O', 'L', 1, 0, 0, 0};
            put(g, gcol_size, 8);
            for (size_t i = 0; i < vl.size(); ++i) {
                put(g, i + 1, 2);
                put(g, 0, 2);
                put(g, 0, 4);
                put(g, vl[i].size(), 8);
                g.insert(g.end(), vl[i].begin(), vl[i].end());
                pad8(g);
            }
            const uint64_t rest = gcol_size - g.size();
            put(g, 0, 2);  // free space object: index 0, size = the rest of the collection
            put(g, 0, 2);
            put(g, 0, 4);
            put(g, rest, 8);
            g.resize(gcol_size, 0);
            emit_at(gcol, g);
        }
        emit(root);
    }
};

extern "C" int igm_h5w_create(const char* path, igm_h5w** out) {
    if (!path || !out) return fail("igm_h5w_create: null argument");
    *out = new igm_h5w();
    (*out)->path = path;
    return 0;
}

extern "C" int igm_h5w_group(igm_h5w* w, const char* path) {
    if (!w) return fail("igm_h5w_group: null writer");
    try {
        const auto parts = split_path(path);
        w->node(parts, parts.size(), true);
        return 0;
    } catch (const Err& e) {
        return fail("igm_h5w_group: %s", e.msg.c_str());
    }
}

extern "C" int igm_h5w_dataset(igm_h5w* w, const char* path, int32_t cls, int32_t size, int32_t is_signed,
                               int32_t rank, const int64_t* dims, const void* data) {
    if (!w || (rank > 0 && !dims)) return fail("igm_h5w_dataset: null argument");
    try {
        if (cls == IGM_H5_VLSTR) raise("use igm_h5w_vlstr for variable-length strings");
        std::vector<uint8_t> dt = dtype_bytes(cls, size, is_signed), ds = space_bytes(rank, dims);
        int64_t n = 1;
        for (int d = 0; d < rank; ++d) n *= dims[d];
        if (n > 0 && !data) raise("no data");
        WNode* d = w->new_leaf(path);
        d->dt = dt;
        d->ds = ds;
        d->data.assign((const uint8_t*)data, (const uint8_t*)data + (size_t)n * size);
        return 0;
    } catch (const Err& e) {
        return fail("igm_h5w_dataset('%s'): %s", path ? path : "", e.msg.c_str());
    }
}

extern "C" int igm_h5w_vlstr(igm_h5w* w, const char* path, const char* attr, const char* str, size_t len) {
    if (!w || (!str && len)) return fail("igm_h5w_vlstr: null argument");
    try {
        const std::string s(str ? str : "", len);
        if (attr) {
            const auto parts = split_path(path);
            WNode* n = w->node(parts, parts.size(), false);
            WAttr a;
            a.name = attr;
            a.dt = dtype_bytes(IGM_H5_VLSTR, 16, 0);
            a.ds = space_bytes(0, nullptr);
            a.vl = true;
            a.vstr = s;
            n->attrs.push_back(a);
        } else {
            WNode* d = w->new_leaf(path);
            d->dt = dtype_bytes(IGM_H5_VLSTR, 16, 0);
            d->ds = space_bytes(0, nullptr);
            d->vl = true;
            d->vstr = s;
        }
        return 0;
    } catch (const Err& e) {
        return fail("igm_h5w_vlstr('%s'): %s", path ? path : "", e.msg.c_str());
    }
}

extern "C" int igm_h5w_attr(igm_h5w* w, const char* path, const char* name, int32_t cls, int32_t size,
                            int32_t is_signed, int32_t rank, const int64_t* dims, const void* data) {
    if (!w || !name || (rank > 0 && !dims)) return fail("igm_h5w_attr: null argument");
    try {
        if (cls == IGM_H5_VLSTR) raise("use igm_h5w_vlstr for variable-length strings");
        const auto parts = split_path(path);
        WNode* n = w->node(parts, parts.size(), false);
        for (auto& a : n->attrs)
            if (a.name == name) raise("attribute '%s' exists", name);
        WAttr a;
        a.name = name;
        a.dt = dtype_bytes(cls, size, is_signed);
        a.ds = space_bytes(rank, dims);
        int64_t ne = 1;
        for (int d = 0; d < rank; ++d) ne *= dims[d];
        if (ne > 0 && !data) raise("no data");
        a.data.assign((const uint8_t*)data, (const uint8_t*)data + (size_t)ne * size);
        if (a.data.size() > 60000) raise("attribute larger than an object header message");
        n->attrs.push_back(a);
        return 0;
    } catch (const Err& e) {
        return fail("igm_h5w_attr('%s', '%s'): %s", path ? path : "", name, e.msg.c_str());
    }
}

extern "C" int igm_h5w_close(igm_h5w* w) {
    if (!w) return fail("igm_h5w_close: null writer");
    std::unique_ptr<igm_h5w> own(w);
    try {
        w->write();
    } catch (const Err& e) {
        return fail("igm_h5w_close('%s'): %s", w->path.c_str(), e.msg.c_str());
    }
    const std::string tmp = w->path + ".part";
    FILE* fp = fopen(tmp.c_str(), "wb");
    if (!fp) return fail("igm_h5w_close: cannot create '%s'", tmp.c_str());
    const size_t n = fwrite(w->out.data(), 1, w->out.size(), fp);
    const int rc = fclose(fp);
    if (n != w->out.size() || rc != 0) {
        remove(tmp.c_str());
        return fail("igm_h5w_close: short write of '%s'", tmp.c_str());
    }
    if (rename(tmp.c_str(), w->path.c_str()) != 0) return fail("igm_h5w_close: cannot rename to '%s'", w->path.c_str());
    return 0;
}

extern "C" int igm_h5w_abort(igm_h5w* w) {
    delete w;
    return 0;
}
