// LSM "replace"-strategy segment reader: restores a flat index from the
// on-disk vectors bucket (PostStartup-style upload straight from segments).
//
// Host-only code, included by runtime.hip (needs wv_index, set_err,
// add_rows_locked).  Format followed:
//  - header (lsmkv/segmentindex/header.go:24-42, ParseHeader :117-134):
//    u16 level, u16 version, u16 secondaryIndices, u16 strategy, u64 indexStart,
//    all little endian; version > CurrentSegmentVersion (=1,
//    header_version.go:15-21) is rejected;
//  - data region [HeaderSize, indexStart) (lsmkv/segment.go:288-289), one
//    replace node after another (segment_serialization.go:34-104 writer,
//    ParseReplaceNode :106-166): u8 tombstone, u64 value length, value,
//    u32 key length, key, then per secondary index u32 length + key;
//  - version >= 1: a trailing CRC32-IEEE over body (bytes after the header,
//    up to size-4) then the header, stored as hash.Sum(nil), i.e. big endian
//    (segment_file.go:274-341, integrity/checksum_reader.go:38,53);
//  - flat's vectors bucket: key = big-endian uint64 doc id, value = d
//    little-endian float32 (flat/index.go:204-208, 317-336).
// Segments are given oldest first, as SegmentGroup orders them; the newest
// entry of a key wins and a tombstone hides the key (replace strategy).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace wvlsm {

static const uint64_t kHeaderSize = 16;    // segmentindex.HeaderSize
static const uint64_t kChecksumSize = 4;   // segmentindex.ChecksumSize
static const uint16_t kCurrentVersion = 1; // segmentindex.CurrentSegmentVersion
static const uint16_t kStrategyReplace = 0;
static const char* kStrategyNames[] = {"replace", "setcollection", "mapcollection",
                                       "roaringset", "roaringsetrange", "inverted"};

struct Mapped {
    const uint8_t* p = nullptr;
    uint64_t size = 0;
    int fd = -1;
    ~Mapped() {
        if (p && size) munmap((void*)p, size);
        if (fd >= 0) close(fd);
    }
};

struct Header {
    uint16_t level, version, secondary, strategy;
    uint64_t index_start;
};

static inline uint16_t le16(const uint8_t* b) { return (uint16_t)(b[0] | (b[1] << 8)); }
static inline uint32_t le32(const uint8_t* b) {
    return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}
static inline uint64_t le64(const uint8_t* b) { return (uint64_t)le32(b) | ((uint64_t)le32(b + 4) << 32); }
static inline uint64_t be64(const uint8_t* b) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | b[i];
    return v;
}

static uint32_t g_crc_table[256];
static std::once_flag g_crc_once;
static uint32_t crc32_update(uint32_t crc, const uint8_t* p, uint64_t n) {
    std::call_once(g_crc_once, [] {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            g_crc_table[i] = c;
        }
    });
    crc = ~crc;
    for (uint64_t i = 0; i < n; i++) crc = g_crc_table[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
    return ~crc;
}

static int map_file(const char* path, Mapped& m) {
    m.fd = open(path, O_RDONLY);
    if (m.fd < 0) return set_err(WV_ERR_INVALID, "open segment %s: %s", path, strerror(errno));
    struct stat st;
    if (fstat(m.fd, &st) != 0) return set_err(WV_ERR_INVALID, "stat segment %s: %s", path, strerror(errno));
    m.size = (uint64_t)st.st_size;
    if (m.size < kHeaderSize)
        return set_err(WV_ERR_INVALID, "parse header: expected %d bytes, got %llu", (int)kHeaderSize,
                       (unsigned long long)m.size);
    void* p = mmap(nullptr, m.size, PROT_READ, MAP_PRIVATE, m.fd, 0);
    if (p == MAP_FAILED) { m.size = 0; return set_err(WV_ERR_INVALID, "mmap file: %s", strerror(errno)); }
    m.p = (const uint8_t*)p;
    return WV_OK;
}

// segment.go:253-272 (ParseHeader, CheckExpectedStrategy, ValidateChecksum)
static int parse_header(const char* path, const Mapped& m, bool validate, Header& h) {
    h.level = le16(m.p);
    h.version = le16(m.p + 2);
    h.secondary = le16(m.p + 4);
    h.strategy = le16(m.p + 6);
    h.index_start = le64(m.p + 8);
    if (h.version > kCurrentVersion) return set_err(WV_ERR_INVALID, "parse header: unsupported version %d", h.version);
    if (h.index_start < kHeaderSize || h.index_start > m.size)
        return set_err(WV_ERR_INVALID, "segment %s: index start %llu outside the file (%llu bytes)", path,
                       (unsigned long long)h.index_start, (unsigned long long)m.size);
    if (validate && h.version >= 1) {
        if (m.size < kHeaderSize + kChecksumSize)
            return set_err(WV_ERR_INVALID, "validate segment \"%s\": read segment file checksum: EOF", path);
        uint32_t crc = crc32_update(0, m.p + kHeaderSize, m.size - kHeaderSize - kChecksumSize);
        crc = crc32_update(crc, m.p, kHeaderSize);
        const uint8_t* s = m.p + m.size - kChecksumSize;
        uint32_t stored = ((uint32_t)s[0] << 24) | ((uint32_t)s[1] << 16) | ((uint32_t)s[2] << 8) | s[3];
        if (crc != stored) return set_err(WV_ERR_INVALID, "validate segment \"%s\": invalid checksum", path);
    }
    return WV_OK;
}

static int check_replace(const Header& h) {
    if (h.strategy != kStrategyReplace) {
        const char* name = h.strategy < 6 ? kStrategyNames[h.strategy] : "n/a";
        return set_err(WV_ERR_UNSUPPORTED,
                       "unsupported strategy in segment: strategy %s (%d) not in expected list [replace]", name,
                       h.strategy);
    }
    return WV_OK;
}

struct Node {
    uint64_t start, end;       // [start, end) of the whole node in the file
    uint64_t value_off, value_len;
    uint64_t key_off;
    uint32_t key_len;
    bool tombstone;
};

// ParseReplaceNode (segment_serialization.go:106-166) over the mmap, bounds-checked
static int parse_node(const Mapped& m, uint64_t pos, uint64_t end, uint16_t secondary, Node& n) {
    n.start = pos;
    if (pos + 9 > end) return set_err(WV_ERR_INVALID, "read tombstone and value length: unexpected EOF at %llu",
                                      (unsigned long long)pos);
    n.tombstone = m.p[pos] == 1;
    n.value_len = le64(m.p + pos + 1);
    pos += 9;
    if (n.value_len > end - pos) return set_err(WV_ERR_INVALID, "read value: unexpected EOF at %llu",
                                                (unsigned long long)pos);
    n.value_off = pos;
    pos += n.value_len;
    if (pos + 4 > end) return set_err(WV_ERR_INVALID, "read key length encoding: unexpected EOF");
    n.key_len = le32(m.p + pos);
    pos += 4;
    if (n.key_len > end - pos) return set_err(WV_ERR_INVALID, "read key: unexpected EOF");
    n.key_off = pos;
    pos += n.key_len;
    for (int j = 0; j < secondary; j++) {
        if (pos + 4 > end) return set_err(WV_ERR_INVALID, "read secondary key length encoding: unexpected EOF");
        uint32_t l = le32(m.p + pos);
        pos += 4;
        if (l > end - pos) return set_err(WV_ERR_INVALID, "read secondary key: unexpected EOF");
        pos += l;
    }
    n.end = pos;
    return WV_OK;
}

}  // namespace wvlsm

extern "C" int wv_lsm_segment_header(const char* path, int32_t validate_checksum, int64_t* out) {
    using namespace wvlsm;
    if (!path || !out) return set_err(WV_ERR_INVALID, "nil argument");
    Mapped m;
    int rc = map_file(path, m);
    if (rc) return rc;
    Header h;
    rc = parse_header(path, m, validate_checksum != 0, h);
    if (rc) return rc;
    out[0] = h.level; out[1] = h.version; out[2] = h.secondary; out[3] = h.strategy;
    out[4] = (int64_t)h.index_start; out[5] = (int64_t)m.size;
    return WV_OK;
}

extern "C" int wv_lsm_segment_scan(const char* path, int32_t validate_checksum, int64_t* node_start,
                                   int64_t* node_end, uint8_t* tombstone, uint64_t* key_id, int64_t cap,
                                   int64_t* out_n) {
    using namespace wvlsm;
    if (!path || !out_n) return set_err(WV_ERR_INVALID, "nil argument");
    Mapped m;
    int rc = map_file(path, m);
    if (rc) return rc;
    Header h;
    rc = parse_header(path, m, validate_checksum != 0, h);
    if (rc) return rc;
    rc = check_replace(h);
    if (rc) return rc;
    int64_t n = 0;
    for (uint64_t pos = kHeaderSize; pos < h.index_start;) {
        Node nd;
        rc = parse_node(m, pos, h.index_start, h.secondary, nd);
        if (rc) return rc;
        if (n < cap) {
            if (node_start) node_start[n] = (int64_t)nd.start;
            if (node_end) node_end[n] = (int64_t)nd.end;
            if (tombstone) tombstone[n] = nd.tombstone ? 1 : 0;
            if (key_id) key_id[n] = nd.key_len == 8 ? be64(m.p + nd.key_off) : ~0ull;
        }
        n++;
        pos = nd.end;
    }
    *out_n = n;
    return WV_OK;
}

// Restore: all segments (oldest first) of flat's vectors bucket into the index.
// out[0] = live vectors uploaded, out[1] = keys hidden by tombstones,
// out[2] = nodes read.  AlreadyIndexed becomes the bucket's live count
// (initBuckets: count = CountAsync, flat/index.go:278-279).
namespace wvlsm {

struct Entry {
    int32_t seg;
    uint64_t value_off, value_len;
    bool tombstone;
};

// every node of the segments (oldest first): the newest entry of each key wins
static int collect(const char* const* paths, int32_t n_paths, bool validate, std::vector<Mapped>& maps,
                   std::unordered_map<uint64_t, Entry>& latest, int64_t& nodes) {
    maps.resize((size_t)std::max(n_paths, 0));
    nodes = 0;
    for (int32_t si = 0; si < n_paths; si++) {
        const char* path = paths[si];
        int rc = map_file(path, maps[si]);
        if (rc) return rc;
        Header h;
        rc = parse_header(path, maps[si], validate, h);
        if (rc) return rc;
        rc = check_replace(h);
        if (rc) return rc;
        for (uint64_t pos = kHeaderSize; pos < h.index_start;) {
            Node nd;
            rc = parse_node(maps[si], pos, h.index_start, h.secondary, nd);
            if (rc) return rc;
            if (nd.key_len != 8)
                return set_err(WV_ERR_INVALID, "segment %s: vectors bucket key of %u bytes (want a big-endian uint64 id)",
                               path, nd.key_len);
            uint64_t id = be64(maps[si].p + nd.key_off);
            latest[id] = Entry{si, nd.value_off, nd.value_len, nd.tombstone};
            nodes++;
            pos = nd.end;
        }
    }
    return WV_OK;
}

// float32SliceFromByteSlice (flat/index.go:331-336) of live[c0, c1) into buf;
// every value must hold d float32 (the first live value fixes d)
static int gather_rows(const char* const* paths, const std::vector<Mapped>& maps,
                       std::unordered_map<uint64_t, Entry>& latest, const std::vector<uint64_t>& live, size_t c0,
                       size_t c1, int64_t d, std::vector<float>& buf) {
    buf.resize((c1 - c0) * (size_t)d);
    for (size_t j = c0; j < c1; j++) {
        const Entry& e = latest[live[j]];
        if ((int64_t)e.value_len != d * 4) {
            return set_err(WV_ERR_INSERT,
                           "insert called with a vector of the wrong size: %lld. Saved length: %lld, path: %s",
                           (long long)(e.value_len / 4), (long long)d, paths[e.seg]);
        }
        memcpy(&buf[(j - c0) * d], maps[e.seg].p + e.value_off, (size_t)d * 4);  // LE host
    }
    return WV_OK;
}

// the vector dimension of a restore: the first live value's float32 count
static int value_dims(std::unordered_map<uint64_t, Entry>& latest, const std::vector<uint64_t>& live, int64_t& d) {
    d = 0;
    if (live.empty()) return WV_OK;
    const Entry& e0 = latest[live[0]];
    if (e0.value_len % 4)
        return set_err(WV_ERR_INVALID, "vector value of %llu bytes is not float32-aligned",
                       (unsigned long long)e0.value_len);
    d = (int64_t)(e0.value_len / 4);
    return WV_OK;
}

static void split_live(std::unordered_map<uint64_t, Entry>& latest, std::vector<uint64_t>& live,
                       std::vector<uint64_t>& dead) {
    live.reserve(latest.size());
    for (auto& kv : latest) (kv.second.tombstone ? dead : live).push_back(kv.first);
    std::sort(live.begin(), live.end());
    std::sort(dead.begin(), dead.end());
}

}  // namespace wvlsm

#ifndef WV_LSM_HOST_ONLY
// Restore: all segments (oldest first) of flat's vectors bucket into the index.
// out[0] = live vectors uploaded, out[1] = keys hidden by tombstones,
// out[2] = nodes read.  AlreadyIndexed becomes the bucket's live count
// (initBuckets: count = CountAsync, flat/index.go:278-279).
extern "C" int wv_index_load_segments(wv_index* idx, const char* const* paths, int32_t n_paths,
                                      int32_t validate_checksum, int64_t* out) {
    using namespace wvlsm;
    if (!idx || (n_paths > 0 && !paths)) return set_err(WV_ERR_INVALID, "nil argument");
    std::vector<Mapped> maps;
    std::unordered_map<uint64_t, Entry> latest;
    int64_t nodes = 0;
    int rc = collect(paths, n_paths, validate_checksum != 0, maps, latest, nodes);
    if (rc) return rc;
    std::vector<uint64_t> live, dead;
    split_live(latest, live, dead);
    if (!dead.empty()) {
        rc = wv_index_delete(idx, dead.data(), (int64_t)dead.size());
        if (rc) return rc;
    }
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    int64_t loaded = 0;
    int64_t d = 0;
    rc = value_dims(latest, live, d);
    if (rc) return rc;
    if (!live.empty()) {
        // the dimension check is ValidateBeforeInsert's (add_rows_locked)
        const int64_t chunk = std::max<int64_t>(1, (256ll << 20) / std::max<int64_t>(d * 4, 1));
        std::vector<float> buf;
        std::vector<uint64_t> ids;
        for (size_t c0 = 0; c0 < live.size(); c0 += (size_t)chunk) {
            size_t c1 = std::min(live.size(), c0 + (size_t)chunk);
            ids.assign(live.begin() + c0, live.begin() + c1);
            rc = gather_rows(paths, maps, latest, live, c0, c1, d, buf);
            if (rc) return rc;
            // the bucket holds the stored bytes (normalised by Add for cosine):
            // upload as they are (PostStartup / restore reads them unchanged)
            rc = add_rows_locked(idx, ids.data(), buf.data(), (int64_t)(c1 - c0), d, true);
            if (rc) return rc;
            loaded += (int64_t)(c1 - c0);
        }
    }
    idx->count = (uint64_t)idx->npresent;
    if (out) { out[0] = loaded; out[1] = (int64_t)dead.size(); out[2] = nodes; }
    return WV_OK;
}
#endif
