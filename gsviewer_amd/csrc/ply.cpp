// Native PLY ingestion and 3dgs row export (include/gsr_io.h).
//
// Ingestion restates the parse half of util_gau.load_ply (util_gau.py:236-305).
// The header is parsed once.  The vertex body is memory-mapped and converted
// column by column into the caller's SoA float32 arrays by a pool of threads,
// each converting a contiguous block of rows.  There is no per-row allocation
// and no per-property dictionary lookup.  The activations stay with the caller
// (gsviewer_amd/ply.py applies the reference's NumPy expressions).
//
// The exporter writes the rows gsconverter keeps in its 3dgs layout
// (base_converter.py:148-170 define_dtype, utility.py:35-65 copy by name,
// main.py:108-110 PlyData.write with native byte order).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "gsr_internal.h"
#include "gsr_io.h"

namespace {

using gsr::set_error;

enum PType { T_I8, T_U8, T_I16, T_U16, T_I32, T_U32, T_F32, T_F64, T_BAD };

int type_size(PType t) {
    switch (t) {
        case T_I8: case T_U8: return 1;
        case T_I16: case T_U16: return 2;
        case T_I32: case T_U32: case T_F32: return 4;
        case T_F64: return 8;
        default: return 0;
    }
}

PType parse_type(const std::string& s) {
    if (s == "char" || s == "int8") return T_I8;
    if (s == "uchar" || s == "uint8") return T_U8;
    if (s == "short" || s == "int16") return T_I16;
    if (s == "ushort" || s == "uint16") return T_U16;
    if (s == "int" || s == "int32") return T_I32;
    if (s == "uint" || s == "uint32") return T_U32;
    if (s == "float" || s == "float32") return T_F32;
    if (s == "double" || s == "float64") return T_F64;
    return T_BAD;
}

struct Prop {
    std::string name;
    PType type = T_BAD;
    int offset = 0;  // byte offset inside a binary row
    bool is_list = false;
};

struct Element {
    std::string name;
    int64_t count = 0;
    std::vector<Prop> props;
    int row_bytes = 0;
    bool has_list = false;
};

struct Header {
    int format = GSR_PLY_BINARY_LE;
    std::vector<Element> elements;
    size_t body_offset = 0;
};

// Header text up to and including "end_header\n".
int parse_header(const char* data, size_t size, Header& h) {
    size_t pos = 0;
    auto next_line = [&](std::string& line) -> bool {
        if (pos >= size) return false;
        size_t e = pos;
        while (e < size && data[e] != '\n') ++e;
        line.assign(data + pos, e - pos);
        if (!line.empty() && line.back() == '\r') line.pop_back();
        pos = e < size ? e + 1 : e;
        return true;
    };
    std::string line;
    if (!next_line(line) || line != "ply") return set_error(GSR_ERR_INVALID, "ply: missing 'ply' magic");
    bool have_format = false, ended = false;
    while (next_line(line)) {
        std::vector<std::string> tok;
        {
            size_t i = 0;
            while (i < line.size()) {
                while (i < line.size() && std::isspace((unsigned char)line[i])) ++i;
                size_t j = i;
                while (j < line.size() && !std::isspace((unsigned char)line[j])) ++j;
                if (j > i) tok.emplace_back(line.substr(i, j - i));
                i = j;
            }
        }
        if (tok.empty()) continue;
        if (tok[0] == "end_header") {
            ended = true;
            break;
        }
        if (tok[0] == "comment" || tok[0] == "obj_info") continue;
        if (tok[0] == "format") {
            if (tok.size() < 2) return set_error(GSR_ERR_INVALID, "ply: bad format line");
            if (tok[1] == "binary_little_endian") h.format = GSR_PLY_BINARY_LE;
            else if (tok[1] == "binary_big_endian") h.format = GSR_PLY_BINARY_BE;
            else if (tok[1] == "ascii") h.format = GSR_PLY_ASCII;
            else return set_error(GSR_ERR_INVALID, "ply: unknown format " + tok[1]);
            have_format = true;
        } else if (tok[0] == "element") {
            if (tok.size() != 3) return set_error(GSR_ERR_INVALID, "ply: bad element line");
            Element e;
            e.name = tok[1];
            char* endp = nullptr;
            e.count = std::strtoll(tok[2].c_str(), &endp, 10);
            if (!endp || *endp || e.count < 0) return set_error(GSR_ERR_INVALID, "ply: bad element count");
            h.elements.push_back(e);
        } else if (tok[0] == "property") {
            if (h.elements.empty()) return set_error(GSR_ERR_INVALID, "ply: property before element");
            Element& e = h.elements.back();
            Prop p;
            if (tok.size() == 5 && tok[1] == "list") {
                p.is_list = true;
                p.name = tok[4];
                e.has_list = true;
            } else if (tok.size() == 3) {
                p.type = parse_type(tok[1]);
                if (p.type == T_BAD) return set_error(GSR_ERR_INVALID, "ply: unknown property type " + tok[1]);
                p.name = tok[2];
                p.offset = e.row_bytes;
                e.row_bytes += type_size(p.type);
            } else {
                return set_error(GSR_ERR_INVALID, "ply: bad property line");
            }
            e.props.push_back(p);
        } else {
            return set_error(GSR_ERR_INVALID, "ply: unexpected header line '" + tok[0] + "'");
        }
    }
    if (!have_format || !ended) return set_error(GSR_ERR_INVALID, "ply: truncated header");
    h.body_offset = pos;
    return GSR_OK;
}

struct MappedFile {
    const char* data = nullptr;
    size_t size = 0;
    int fd = -1;
    ~MappedFile() {
        if (data && data != MAP_FAILED) munmap(const_cast<char*>(data), size);
        if (fd >= 0) close(fd);
    }
    int open_read(const char* path) {
        fd = ::open(path, O_RDONLY);
        if (fd < 0) return set_error(GSR_ERR_INVALID, std::string("ply: cannot open ") + path + ": " + strerror(errno));
        struct stat st;
        if (fstat(fd, &st) != 0) return set_error(GSR_ERR_INVALID, "ply: fstat failed");
        size = (size_t)st.st_size;
        if (size == 0) return set_error(GSR_ERR_INVALID, "ply: empty file");
        void* p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (p == MAP_FAILED) return set_error(GSR_ERR_INVALID, "ply: mmap failed");
        data = static_cast<const char*>(p);
        madvise(p, size, MADV_SEQUENTIAL);
        return GSR_OK;
    }
};

// The vertex element, where it starts in the body, and the columns load_ply uses.
struct Layout {
    Header h;
    int vi = -1;               // index of the vertex element
    size_t vertex_offset = 0;  // byte offset of its first row (binary)
    int64_t skip_lines = 0;    // ascii: body lines before the first vertex row
    int xyz[3], op, dc[3], scale[3], rot[4];
    std::vector<int> rest;     // f_rest_* property indices sorted by suffix
    int sh_dim = 3;
};

bool suffix_int(const std::string& name, long& v) {
    const size_t u = name.rfind('_');
    const std::string s = u == std::string::npos ? name : name.substr(u + 1);
    if (s.empty()) return false;
    char* endp = nullptr;
    v = std::strtol(s.c_str(), &endp, 10);
    return endp && *endp == 0;
}

// Names starting with `prefix`, sorted by int(name.split('_')[-1]) (util_gau.py:262-273).
int sorted_by_suffix(const Element& e, const char* prefix, std::vector<int>& out) {
    std::vector<std::pair<long, int>> v;
    for (int i = 0; i < (int)e.props.size(); ++i) {
        if (e.props[i].name.rfind(prefix, 0) != 0) continue;
        long k;
        if (!suffix_int(e.props[i].name, k))
            return set_error(GSR_ERR_INVALID, "ply: property '" + e.props[i].name + "' has no integer suffix");
        v.emplace_back(k, i);
    }
    std::stable_sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.first < b.first; });
    out.clear();
    for (auto& p : v) out.push_back(p.second);
    return GSR_OK;
}

int find_prop(const Element& e, const char* name) {
    for (int i = 0; i < (int)e.props.size(); ++i)
        if (e.props[i].name == name) return i;
    return -1;
}

// Header + where the vertex rows start (all that the row writer needs).
int locate_vertex(const MappedFile& f, Layout& L) {
    int rc = parse_header(f.data, f.size, L.h);
    if (rc) return rc;
    size_t off = L.h.body_offset;
    int64_t lines = 0;
    for (int i = 0; i < (int)L.h.elements.size(); ++i) {
        const Element& e = L.h.elements[i];
        if (e.name == "vertex") {
            L.vi = i;
            break;
        }
        if (L.h.format == GSR_PLY_ASCII) {
            lines += e.count;
        } else {
            if (e.has_list) return set_error(GSR_ERR_INVALID, "ply: list element before 'vertex' is not supported");
            off += (size_t)e.count * (size_t)e.row_bytes;
        }
    }
    if (L.vi < 0) return set_error(GSR_ERR_INVALID, "ply: no 'vertex' element");
    const Element& v = L.h.elements[L.vi];
    if (v.has_list) return set_error(GSR_ERR_INVALID, "ply: list property in the vertex element");
    L.vertex_offset = off;
    L.skip_lines = lines;
    if (L.h.format != GSR_PLY_ASCII && off + (size_t)v.count * (size_t)v.row_bytes > f.size)
        return set_error(GSR_ERR_INVALID, "ply: file shorter than its header says");
    return GSR_OK;
}

// locate_vertex + the columns load_ply reads (util_gau.py:241-293).
int make_layout(const MappedFile& f, Layout& L) {
    int rc = locate_vertex(f, L);
    if (rc) return rc;
    const Element& v = L.h.elements[L.vi];
    static const char* xyz[3] = {"x", "y", "z"};
    static const char* dc[3] = {"f_dc_0", "f_dc_1", "f_dc_2"};
    for (int k = 0; k < 3; ++k) {
        if ((L.xyz[k] = find_prop(v, xyz[k])) < 0) return set_error(GSR_ERR_INVALID, std::string("ply: no property ") + xyz[k]);
        if ((L.dc[k] = find_prop(v, dc[k])) < 0) return set_error(GSR_ERR_INVALID, std::string("ply: no property ") + dc[k]);
    }
    if ((L.op = find_prop(v, "opacity")) < 0) return set_error(GSR_ERR_INVALID, "ply: no property opacity");
    std::vector<int> sc, ro;
    if ((rc = sorted_by_suffix(v, "f_rest_", L.rest))) return rc;
    if ((rc = sorted_by_suffix(v, "scale_", sc))) return rc;
    if ((rc = sorted_by_suffix(v, "rot", ro))) return rc;
    if (!L.rest.empty() && L.rest.size() != 45)
        return set_error(GSR_ERR_INVALID, "ply: " + std::to_string(L.rest.size()) +
                                              " f_rest_* properties; load_ply reshapes them to (N, 3, 15)");
    if (sc.size() != 3) return set_error(GSR_ERR_INVALID, "ply: expected 3 scale_* properties");
    if (ro.size() != 4) return set_error(GSR_ERR_INVALID, "ply: expected 4 rot* properties");
    for (int k = 0; k < 3; ++k) L.scale[k] = sc[k];
    for (int k = 0; k < 4; ++k) L.rot[k] = ro[k];
    L.sh_dim = L.rest.empty() ? 3 : 48;
    return GSR_OK;
}

template <typename T>
inline T load_swapped(const char* p, bool swap) {
    T v;
    std::memcpy(&v, p, sizeof(T));
    if (swap) {
        unsigned char b[sizeof(T)];
        std::memcpy(b, &v, sizeof(T));
        std::reverse(b, b + sizeof(T));
        std::memcpy(&v, b, sizeof(T));
    }
    return v;
}

inline float read_as_float(const char* p, PType t, bool swap) {
    switch (t) {
        case T_I8: return (float)*reinterpret_cast<const int8_t*>(p);
        case T_U8: return (float)*reinterpret_cast<const uint8_t*>(p);
        case T_I16: return (float)load_swapped<int16_t>(p, swap);
        case T_U16: return (float)load_swapped<uint16_t>(p, swap);
        case T_I32: return (float)load_swapped<int32_t>(p, swap);
        case T_U32: return (float)load_swapped<uint32_t>(p, swap);
        case T_F32: return load_swapped<float>(p, swap);
        case T_F64: return (float)load_swapped<double>(p, swap);
        default: return 0.f;
    }
}

// One destination column: property -> dst[row * stride + col].
struct Column {
    int prop;
    float* dst;
    int stride, col;
};

std::vector<Column> columns(const Layout& L, float* xyz, float* rot, float* scale, float* opacity, float* sh) {
    std::vector<Column> c;
    for (int k = 0; k < 3; ++k) c.push_back({L.xyz[k], xyz, 3, k});
    for (int k = 0; k < 4; ++k) c.push_back({L.rot[k], rot, 4, k});
    for (int k = 0; k < 3; ++k) c.push_back({L.scale[k], scale, 3, k});
    c.push_back({L.op, opacity, 1, 0});
    for (int k = 0; k < 3; ++k) c.push_back({L.dc[k], sh, L.sh_dim, k});
    // f_rest reshaped (3, 15) then transposed: f_rest[ch*15 + j] -> sh[3 + 3j + ch]
    for (int r = 0; r < (int)L.rest.size(); ++r) c.push_back({L.rest[r], sh, L.sh_dim, 3 + 3 * (r % 15) + r / 15});
    return c;
}

// The same columns into flat rows [xyz, rot, scale, opacity, sh] (util_gau.py:40-42).
std::vector<Column> flat_columns(const Layout& L, float* flat) {
    const int rec = 11 + L.sh_dim;
    std::vector<Column> c;
    for (int k = 0; k < 3; ++k) c.push_back({L.xyz[k], flat, rec, k});
    for (int k = 0; k < 4; ++k) c.push_back({L.rot[k], flat, rec, 3 + k});
    for (int k = 0; k < 3; ++k) c.push_back({L.scale[k], flat, rec, 7 + k});
    c.push_back({L.op, flat, rec, 10});
    for (int k = 0; k < 3; ++k) c.push_back({L.dc[k], flat, rec, 11 + k});
    for (int r = 0; r < (int)L.rest.size(); ++r) c.push_back({L.rest[r], flat, rec, 11 + 3 + 3 * (r % 15) + r / 15});
    return c;
}

int threads_for(int32_t n_threads, int64_t rows) {
    int t = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
    const int64_t min_rows = 16384;  // below this a thread costs more than it converts
    t = (int)std::min<int64_t>(t, std::max<int64_t>(1, rows / min_rows));
    return std::max(1, t);
}

template <typename F>
void parallel_rows(int64_t n, int nt, F&& fn) {
    if (nt <= 1) {
        fn(0, n);
        return;
    }
    std::vector<std::thread> pool;
    const int64_t per = (n + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const int64_t a = t * per, b = std::min(n, a + per);
        if (a >= b) break;
        pool.emplace_back([&fn, a, b] { fn(a, b); });
    }
    for (auto& th : pool) th.join();
}

// ascii: row r's values as floats (tokens in property order).
int read_ascii(const MappedFile& f, const Layout& L, const std::vector<Column>& cols) {
    const Element& v = L.h.elements[L.vi];
    size_t pos = L.h.body_offset;
    auto skip_line = [&]() {
        while (pos < f.size && f.data[pos] != '\n') ++pos;
        if (pos < f.size) ++pos;
    };
    for (int64_t i = 0; i < L.skip_lines; ++i) skip_line();
    std::vector<float> vals(v.props.size());
    for (int64_t r = 0; r < v.count; ++r) {
        for (size_t p = 0; p < v.props.size(); ++p) {
            while (pos < f.size && (f.data[pos] == ' ' || f.data[pos] == '\t' || f.data[pos] == '\r' || f.data[pos] == '\n')) ++pos;
            if (pos >= f.size) return set_error(GSR_ERR_INVALID, "ply: ascii body truncated");
            char buf[64];
            size_t k = 0;
            while (pos < f.size && !std::isspace((unsigned char)f.data[pos]) && k < sizeof(buf) - 1) buf[k++] = f.data[pos++];
            buf[k] = 0;
            char* endp = nullptr;
            const double d = std::strtod(buf, &endp);
            if (endp == buf) return set_error(GSR_ERR_INVALID, "ply: bad ascii value");
            vals[p] = (float)d;
        }
        for (const Column& c : cols) c.dst[r * c.stride + c.col] = vals[c.prop];
    }
    return GSR_OK;
}

}  // namespace

extern "C" int gsr_ply_probe(const char* path, gsr_ply_info* info) {
    if (!path || !info) return set_error(GSR_ERR_INVALID, "ply_probe: null argument");
    MappedFile f;
    int rc = f.open_read(path);
    if (rc) return rc;
    Layout L;
    if ((rc = make_layout(f, L))) return rc;
    const Element& v = L.h.elements[L.vi];
    info->n = v.count;
    info->sh_dim = L.sh_dim;
    info->format = L.h.format;
    info->n_properties = (int32_t)v.props.size();
    info->row_bytes = L.h.format == GSR_PLY_ASCII ? 0 : v.row_bytes;
    info->body_offset = (int64_t)L.vertex_offset;
    return GSR_OK;
}

extern "C" int gsr_ply_read(const char* path, float* xyz, float* rot, float* scale, float* opacity, float* sh,
                            int32_t n_threads) {
    if (!path || !xyz || !rot || !scale || !opacity || !sh) return set_error(GSR_ERR_INVALID, "ply_read: null argument");
    MappedFile f;
    int rc = f.open_read(path);
    if (rc) return rc;
    Layout L;
    if ((rc = make_layout(f, L))) return rc;
    const Element& v = L.h.elements[L.vi];
    const std::vector<Column> cols = columns(L, xyz, rot, scale, opacity, sh);
    if (L.h.format == GSR_PLY_ASCII) return read_ascii(f, L, cols);
    const bool swap = L.h.format == GSR_PLY_BINARY_BE;
    const char* base = f.data + L.vertex_offset;
    const int rb = v.row_bytes;
    // per column: (byte offset, type) resolved once
    std::vector<std::pair<int, PType>> src(cols.size());
    for (size_t c = 0; c < cols.size(); ++c) src[c] = {v.props[cols[c].prop].offset, v.props[cols[c].prop].type};
    parallel_rows(v.count, threads_for(n_threads, v.count), [&](int64_t a, int64_t b) {
        for (int64_t r = a; r < b; ++r) {
            const char* row = base + r * rb;
            for (size_t c = 0; c < cols.size(); ++c)
                cols[c].dst[r * cols[c].stride + cols[c].col] = read_as_float(row + src[c].first, src[c].second, swap);
        }
    });
    return GSR_OK;
}

namespace gsr {

// Raw vertex rows streamed to the device: chunks of kChunkRows rows are
// converted by the thread pool into one of two pinned buffers and copied
// asynchronously on `s` while the next chunk is converted (an event per
// buffer guards its reuse).  ASCII bodies are parsed whole, then copied.
int ply_stream_flat(const char* path, int32_t n_threads, hipStream_t s, float** flat_dev, int64_t* n_out,
                    int32_t* sh_dim_out) {
    *flat_dev = nullptr;
    MappedFile f;
    int rc = f.open_read(path);
    if (rc) return rc;
    Layout L;
    if ((rc = make_layout(f, L))) return rc;
    const Element& v = L.h.elements[L.vi];
    const int64_t n = v.count;
    const int rec = 11 + L.sh_dim;
    *n_out = n;
    *sh_dim_out = L.sh_dim;
    float* dev = nullptr;
    if (hipMalloc(&dev, (size_t)std::max<int64_t>(n, 1) * rec * sizeof(float)) != hipSuccess)
        return set_error(GSR_ERR_NOMEM, "ply: hipMalloc of the row buffer failed");
    constexpr int64_t kChunkRows = 1 << 17;
    const int64_t chunk = L.h.format == GSR_PLY_ASCII ? std::max<int64_t>(n, 1) : std::min<int64_t>(kChunkRows, std::max<int64_t>(n, 1));
    float* pin[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    auto cleanup = [&](int code) {
        for (int b = 0; b < 2; ++b) {
            if (done[b]) {
                (void)hipEventSynchronize(done[b]);
                (void)hipEventDestroy(done[b]);
            }
            if (pin[b]) (void)hipHostFree(pin[b]);
        }
        if (code != GSR_OK) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(dev);
        } else {
            *flat_dev = dev;
        }
        return code;
    };
    const int nbuf = L.h.format == GSR_PLY_ASCII ? 1 : 2;
    for (int b = 0; b < nbuf; ++b) {
        if (hipHostMalloc(&pin[b], (size_t)chunk * rec * sizeof(float), hipHostMallocDefault) != hipSuccess)
            return cleanup(set_error(GSR_ERR_NOMEM, "ply: pinned staging allocation failed"));
        if (hipEventCreateWithFlags(&done[b], hipEventDisableTiming) != hipSuccess)
            return cleanup(set_error(GSR_ERR_HIP, "ply: event creation failed"));
    }
    if (n == 0) return cleanup(GSR_OK);
    if (L.h.format == GSR_PLY_ASCII) {
        if ((rc = read_ascii(f, L, flat_columns(L, pin[0])))) return cleanup(rc);
        if (hipMemcpyAsync(dev, pin[0], (size_t)n * rec * sizeof(float), hipMemcpyHostToDevice, s) != hipSuccess)
            return cleanup(set_error(GSR_ERR_HIP, "ply: host-to-device copy failed"));
        return cleanup(GSR_OK);
    }
    const bool swap = L.h.format == GSR_PLY_BINARY_BE;
    const int rb = v.row_bytes;
    const int nt = threads_for(n_threads, chunk);
    for (int64_t r0 = 0, k = 0; r0 < n; r0 += chunk, ++k) {
        const int b = (int)(k & 1);
        const int64_t m = std::min(chunk, n - r0);
        if (k >= 2 && hipEventSynchronize(done[b]) != hipSuccess)  // its previous copy has left the buffer
            return cleanup(set_error(GSR_ERR_HIP, "ply: staging copy failed"));
        const std::vector<Column> cols = flat_columns(L, pin[b]);
        std::vector<std::pair<int, PType>> src(cols.size());
        for (size_t c = 0; c < cols.size(); ++c) src[c] = {v.props[cols[c].prop].offset, v.props[cols[c].prop].type};
        const char* base = f.data + L.vertex_offset + (size_t)r0 * rb;
        parallel_rows(m, std::min<int>(nt, std::max<int64_t>(1, m / 16384)), [&](int64_t a, int64_t e) {
            for (int64_t r = a; r < e; ++r) {
                const char* row = base + r * rb;
                for (size_t c = 0; c < cols.size(); ++c)
                    cols[c].dst[r * cols[c].stride + cols[c].col] = read_as_float(row + src[c].first, src[c].second, swap);
            }
        });
        if (hipMemcpyAsync(dev + r0 * rec, pin[b], (size_t)m * rec * sizeof(float), hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            hipEventRecord(done[b], s) != hipSuccess)
            return cleanup(set_error(GSR_ERR_HIP, "ply: host-to-device copy failed"));
    }
    return cleanup(GSR_OK);
}

}  // namespace gsr

extern "C" int gsr_ply_write_3dgs(const char* in_path, const char* out_path, const int64_t* rows, int64_t n_rows,
                                  int32_t n_threads) {
    if (!in_path || !out_path) return set_error(GSR_ERR_INVALID, "ply_write_3dgs: null path");
    MappedFile f;
    int rc = f.open_read(in_path);
    if (rc) return rc;
    Layout L;
    if ((rc = locate_vertex(f, L))) return rc;
    if (L.h.format == GSR_PLY_ASCII) return set_error(GSR_ERR_INVALID, "ply_write_3dgs: ascii input not supported");
    const Element& v = L.h.elements[L.vi];
    if (!rows) n_rows = v.count;
    if (n_rows < 0 || n_rows > v.count) return set_error(GSR_ERR_INVALID, "ply_write_3dgs: bad row count");
    if (rows)
        for (int64_t i = 0; i < n_rows; ++i)
            if (rows[i] < 0 || rows[i] >= v.count || (i && rows[i] <= rows[i - 1]))
                return set_error(GSR_ERR_INVALID, "ply_write_3dgs: rows must be ascending and in range");

    // gsconverter's 3dgs dtype (base_converter.py:154-162)
    std::vector<std::string> names = {"x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"};
    for (int i = 0; i < 45; ++i) names.push_back("f_rest_" + std::to_string(i));
    names.push_back("opacity");
    for (int i = 0; i < 3; ++i) names.push_back("scale_" + std::to_string(i));
    for (int i = 0; i < 4; ++i) names.push_back("rot_" + std::to_string(i));
    const int n_out = (int)names.size();
    // source property of each output field: copy by name, else by stripping a
    // gsconverter prefix; a later source field overwrites an earlier match
    // (utility.py:43-65 iterates the source fields in order)
    std::vector<int> from(n_out, -1);
    static const char* prefixes[] = {"scal_", "scalar_", "scalar_scal_"};
    for (int p = 0; p < (int)v.props.size(); ++p) {
        const std::string& nm = v.props[p].name;
        auto it = std::find(names.begin(), names.end(), nm);
        if (it == names.end())
            for (const char* pre : prefixes)
                if (nm.rfind(pre, 0) == 0) {
                    it = std::find(names.begin(), names.end(), nm.substr(std::strlen(pre)));
                    if (it != names.end()) break;
                }
        if (it != names.end()) from[it - names.begin()] = p;
    }

    std::string hdr = "ply\nformat binary_little_endian 1.0\nelement vertex " + std::to_string(n_rows) + "\n";
    for (auto& nm : names) hdr += "property float " + nm + "\n";
    hdr += "end_header\n";
    const size_t out_row = (size_t)n_out * 4;
    std::vector<float> body((size_t)n_rows * n_out);
    const bool swap = L.h.format == GSR_PLY_BINARY_BE;
    const char* base = f.data + L.vertex_offset;
    parallel_rows(n_rows, threads_for(n_threads, n_rows), [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            const char* row = base + (rows ? rows[i] : i) * (int64_t)v.row_bytes;
            float* o = body.data() + (size_t)i * n_out;
            for (int k = 0; k < n_out; ++k)
                o[k] = from[k] < 0 ? 0.f : read_as_float(row + v.props[from[k]].offset, v.props[from[k]].type, swap);
        }
    });
    FILE* fo = std::fopen(out_path, "wb");
    if (!fo) return set_error(GSR_ERR_INVALID, std::string("ply_write_3dgs: cannot create ") + out_path);
    bool ok = std::fwrite(hdr.data(), 1, hdr.size(), fo) == hdr.size();
    ok = ok && (n_rows == 0 || std::fwrite(body.data(), out_row, (size_t)n_rows, fo) == (size_t)n_rows);
    ok = (std::fclose(fo) == 0) && ok;
    if (!ok) return set_error(GSR_ERR_INVALID, std::string("ply_write_3dgs: write failed for ") + out_path);
    return GSR_OK;
}
