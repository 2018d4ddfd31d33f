// Host-only ASan/UBSan fuzz harness of the LSM segment reader
// (weaviate_amd/csrc/lsm_segment.hip): the reference's own segment files
// (tests/golden/lsm) and written variants are mutated -- truncation, byte
// flips, huge / off-by-one length fields, moved index start, bad checksums --
// and every mutant goes through header parsing, the node scan and the restore
// path's collect + row gather.  Any out-of-bounds read aborts (ASan); errors
// must come back as WV_ERR_* codes.  Build + run: tools/asan_lsm.sh.
#include <cerrno>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "../include/wv_knn.h"

static thread_local std::string g_err;
static int set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define WV_LSM_HOST_ONLY
#include "../weaviate_amd/csrc/lsm_segment.hip"

static std::vector<uint8_t> read_file(const char* p) {
    std::vector<uint8_t> b;
    FILE* f = fopen(p, "rb");
    if (!f) return b;
    fseek(f, 0, SEEK_END);
    b.resize((size_t)ftell(f));
    fseek(f, 0, SEEK_SET);
    if (fread(b.data(), 1, b.size(), f) != b.size()) b.clear();
    fclose(f);
    return b;
}

static void write_file(const char* p, const std::vector<uint8_t>& b) {
    FILE* f = fopen(p, "wb");
    if (!f) return;
    fwrite(b.data(), 1, b.size(), f);
    fclose(f);
}

static void put_le(std::vector<uint8_t>& b, size_t pos, uint64_t v, int n) {
    for (int i = 0; i < n && pos + i < b.size(); i++) b[pos + i] = (uint8_t)(v >> (8 * i));
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: lsm_fuzz <tmpdir> <iterations> <seed files...>\n");
        return 2;
    }
    const std::string tmp = argv[1];
    const long iters = atol(argv[2]);
    std::vector<std::vector<uint8_t>> seeds;
    for (int i = 3; i < argc; i++) {
        auto b = read_file(argv[i]);
        if (!b.empty()) seeds.push_back(b);
    }
    if (seeds.empty()) return 2;
    std::mt19937_64 rng(12345);
    long ok = 0, err = 0;
    std::vector<int64_t> ns(4096), ne(4096);
    std::vector<uint8_t> tb(4096);
    std::vector<uint64_t> ki(4096);
    for (long it = 0; it < iters; it++) {
        std::vector<uint8_t> b = seeds[rng() % seeds.size()];
        const int nm = 1 + (int)(rng() % 4);
        for (int m = 0; m < nm && !b.empty(); m++) {
            switch (rng() % 7) {
            case 0: b.resize(rng() % (b.size() + 1)); break;                                   // truncate
            case 1: b[rng() % b.size()] ^= (uint8_t)(1u << (rng() % 8)); break;               // bit flip
            case 2: put_le(b, 16 + rng() % std::max<size_t>(b.size(), 1), rng(), 8); break;   // random u64 (lengths)
            case 3: put_le(b, 16 + rng() % std::max<size_t>(b.size(), 1), (uint64_t)-1 - (rng() % 16), 8); break;
            case 4: put_le(b, 8, rng() % (b.size() + 64), 8); break;                          // index start
            case 5: put_le(b, 2, rng() % 3, 2); break;                                        // version
            default: put_le(b, 4, rng() % 4, 2); break;                                       // secondary indices
            }
        }
        const std::string path = tmp + "/mut.db";
        write_file(path.c_str(), b);
        for (int v = 0; v < 2; v++) {
            int64_t hdr[6];
            int rc = wv_lsm_segment_header(path.c_str(), v, hdr);
            int64_t n = 0;
            rc |= wv_lsm_segment_scan(path.c_str(), v, ns.data(), ne.data(), tb.data(), ki.data(), (int64_t)ns.size(), &n);
            // restore path: collect + gather (no device)
            const char* paths[2] = {path.c_str(), path.c_str()};
            std::vector<wvlsm::Mapped> maps;
            std::unordered_map<uint64_t, wvlsm::Entry> latest;
            int64_t nodes = 0;
            int rc2 = wvlsm::collect(paths, 2, v != 0, maps, latest, nodes);
            if (!rc2) {
                std::vector<uint64_t> live, dead;
                wvlsm::split_live(latest, live, dead);
                int64_t d = 0;
                rc2 = wvlsm::value_dims(latest, live, d);
                if (!rc2 && !live.empty() && d > 0 && d < (1 << 20)) {
                    std::vector<float> buf;
                    rc2 = wvlsm::gather_rows(paths, maps, latest, live, 0, live.size(), d, buf);
                }
            }
            if (rc || rc2) err++; else ok++;
            if ((rc && rc > 0) || (rc2 && rc2 > 0)) { fprintf(stderr, "positive return code\n"); return 1; }
        }
    }
    printf("lsm_fuzz: %ld iterations, %ld parses ok, %ld rejected with an error\n", iters, ok, err);
    return 0;
}
