// kc_cli.cpp -- `kaarme` drop-in command line on top of libkc.so.
//
// Same interface as the reference's main.cpp:127-156 (CLI11 options, exactly one
// of -s/-u, -u needs -b, -f needs -b), the same input format detection
// (main.cpp:19-68), the same chunking (kc_plan_chunks == io_worker +
// read_chunk_from_file) and the same output text ("<CANONICAL_KMER> <count>\n" for
// T(c) >= a, default file "<input stem>.kaarme_counts", main.cpp:189-191).
// Exit codes of option errors follow CLI11's ExitCodes (CLI11.hpp).
//
// Deliberate differences (documented in DESIGN.md): -t defaults to 3 (the reference
// crashes without it); gzip input is decompressed completely (the reference
// truncates it); the work runs on one MI355X.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kc_api.h"

namespace {

enum CliExit { kConversion = 104, kValidation = 105, kRequired = 106, kRequires = 107, kExtras = 109 };

struct Args {
    std::string input, output;
    long long k = 0;
    int mode = 2;
    unsigned long long min_abundance = 2;
    int threads = 3;
    bool use_bf = false;
    double fpr = 0.01;
    bool fpr_set = false;
    bool have_s = false, have_u = false;
    unsigned long long slots = 0, unique = 0;
    int device = 0;
    std::string gunzip_to;  // test hook: write the decompressed input there and exit (no GPU)
    // extensions, not in --help: --host-chunks stages host chunks instead of one
    // device image; --no-warmup skips the untimed warm-up pass; --readers N upload threads; --phases
    // prints the counting pass's phase times on stderr; --digest-only prints the output's digest
    // (kc_output_digest) instead of writing it; --table-sizing auto|s|estimate: the device table from
    // -s or from the input's distinct estimate (auto: the estimate when the -s table passes 16 GiB)
    bool host_chunks = false, no_warmup = false, phases = false, digest_only = false;
    int table_sizing = 0;  // --table-sizing auto (0) | s (1) | estimate (2)
    unsigned readers = 1;
};

void usage(const char* prog) {
    std::cout << "Space-efficient k-mer counter\n"
                 "Usage: " << prog << " [OPTIONS] INPUT KLEN\n\n"
                 "Positionals:\n"
                 "  INPUT TEXT:FILE REQUIRED    Input file (automatic format detection)\n"
                 "  KLEN INT REQUIRED           k-mer length\n\n"
                 "Options:\n"
                 "  -h,--help                   Print this help message and exit\n"
                 "  -m,--hash-table-type INT    Hash table type: 0 for plain and 2 for kaarme (def. 2)\n"
                 "  -a,--min-k-abu UINT         Minimum abundance threshold for the output k-mers (def. 2)\n"
                 "  -t,--threads UINT           Number of working threads (def. 3)\n"
                 "  -o,--output-file TEXT       Output file where the k-mer counts will be stored\n"
                 "  -b,--use-bfilter            Use bloom filters to discard unique k-mers\n"
                 "  -f,--bfilter-fpr FLOAT      Bloom filter false positive rate (def. 0.01)\n"
                 "  --device INT                HIP device ordinal (def. 0)\n"
                 "  --strict-capacity           fail like the reference once the distinct k-mers pass its table\n"
                 "                              size next_prime3mod4(-s) (the device table keeps 25 % headroom)\n\n"
                 "Mandatory params:\n"
                 "  -s,--hash-tab-size UINT     Hash table size\n"
                 "  -u,--unq-kmers UINT         Estimated number of unique k-mers\n";
}

int cli_error(int code, const std::string& msg) {
    std::cerr << msg << "\nRun with --help for more information.\n";
    return code;
}

bool parse_uint(const std::string& s, unsigned long long* v) {
    if (s.empty() || s[0] == '-' || s[0] == '+') return false;
    char* end = nullptr;
    errno = 0;
    *v = std::strtoull(s.c_str(), &end, 10);
    return errno == 0 && end && *end == 0;
}
bool parse_int(const std::string& s, long long* v) {
    if (s.empty()) return false;
    char* end = nullptr;
    errno = 0;
    *v = std::strtoll(s.c_str(), &end, 10);
    return errno == 0 && end && *end == 0;
}
bool parse_double(const std::string& s, double* v) {
    if (s.empty()) return false;
    char* end = nullptr;
    *v = std::strtod(s.c_str(), &end);
    return end && *end == 0;
}

// BGZF input (blocked gzip, bgzip / htslib: every member carries its compressed size in a
// 'BC' extra subfield and is at most 64 KiB uncompressed): the members are inflated by up to
// `nt` threads straight into their slots of one buffer (each member's ISIZE gives its slot).
// Returns false when the file is not BGZF (the caller reads it as one stream); *bad is set
// when a member does not inflate to its ISIZE (corrupt input).
static bool gunzip_bgzf(const uint8_t* z, uint64_t n, int nt, std::vector<uint8_t>* out, bool* bad) {
    std::vector<uint64_t> off, len, dst;
    std::vector<uint32_t> usz;
    uint64_t p = 0, total = 0;
    while (p < n) {
        if (n - p < 28 || z[p] != 0x1f || z[p + 1] != 0x8b || z[p + 2] != 8 || !(z[p + 3] & 4)) return false;
        const uint32_t xlen = z[p + 10] | (uint32_t)z[p + 11] << 8;
        if (12 + (uint64_t)xlen > n - p) return false;
        uint64_t bsize = 0;
        for (uint32_t q = 0; q + 4 <= xlen;) {
            const uint8_t* f = z + p + 12 + q;
            const uint32_t sl = f[2] | (uint32_t)f[3] << 8;
            if (f[0] == 'B' && f[1] == 'C' && sl == 2 && q + 6 <= xlen) {
                bsize = (f[4] | (uint32_t)f[5] << 8) + 1ULL;
                break;
            }
            q += 4 + sl;
        }
        if (bsize < 20 + (uint64_t)xlen || bsize > n - p) return false;
        const uint8_t* t = z + p + bsize - 4;
        const uint32_t isz = t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24;
        if (isz > 65536) {  // a BGZF member holds at most 64 KiB: a forged or corrupt ISIZE
            *bad = true;
            return true;
        }
        off.push_back(p);
        len.push_back(bsize);
        usz.push_back(isz);
        dst.push_back(total);
        total += isz;
        p += bsize;
    }
    if (off.size() < 2) return false;  // one member: nothing to split
    try {
        out->resize(total);
    } catch (const std::bad_alloc&) {
        *bad = true;
        return true;
    }
    std::atomic<uint64_t> next{0};
    std::atomic<bool> fail{false};
    auto work = [&]() {
        uint8_t dummy = 0;
        for (uint64_t i; (i = next.fetch_add(1)) < off.size() && !fail.load();) {
            z_stream st{};
            if (inflateInit2(&st, 16 + MAX_WBITS) != Z_OK) { fail = true; break; }
            st.next_in = const_cast<Bytef*>(z + off[i]);
            st.avail_in = (uInt)len[i];
            st.next_out = usz[i] ? out->data() + dst[i] : &dummy;
            st.avail_out = usz[i] ? usz[i] : 1;
            const int r = inflate(&st, Z_FINISH);
            if (r != Z_STREAM_END || st.total_out != usz[i] || st.avail_in != 0) fail = true;
            inflateEnd(&st);
        }
    };
    const int T = std::max(1, std::min<int>(nt, (int)std::min<uint64_t>(off.size(), 64)));
    std::vector<std::thread> th;
    for (int i = 1; i < T; i++) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
    *bad = fail.load();
    return true;
}

// returns -1 on success, else exit code
int parse(int argc, char** argv, Args* a) {
    std::vector<std::string> pos;
    for (int i = 1; i < argc; i++) {
        std::string o = argv[i];
        std::string val;
        bool has_inline = false;
        if (o.rfind("--", 0) == 0 && o.find('=') != std::string::npos) {
            val = o.substr(o.find('=') + 1);
            o = o.substr(0, o.find('='));
            has_inline = true;
        }
        auto next = [&](std::string* out) -> bool {
            if (has_inline) { *out = val; return true; }
            if (i + 1 >= argc) return false;
            *out = argv[++i];
            return true;
        };
        if (o == "-h" || o == "--help") { usage(argv[0]); return 0; }
        if (o == "-b" || o == "--use-bfilter") { a->use_bf = true; continue; }
        if (o == "--strict-capacity") { setenv("KC_STRICT_CAPACITY", "1", 1); continue; }  // kc_api.h
        if (o == "--host-chunks") { a->host_chunks = true; continue; }
        if (o == "--no-warmup") { a->no_warmup = true; continue; }
        if (o == "--phases") { a->phases = true; continue; }
        if (o == "--digest-only") { a->digest_only = true; continue; }
        if (o.size() > 1 && o[0] == '-' && !(o.size() > 1 && std::isdigit((unsigned char)o[1]))) {
            std::string v;
            if (!next(&v)) return cli_error(kRequired, o + " requires an argument");
            unsigned long long u;
            long long si;
            double d;
            if (o == "-m" || o == "--hash-table-type") {
                if (!parse_int(v, &si)) return cli_error(kConversion, "Could not convert: " + o + " = " + v);
                if (si < 0 || si > 2) return cli_error(kValidation, o + ": Value " + v + " not in range 0 to 2");
                a->mode = (int)si;
            } else if (o == "-a" || o == "--min-k-abu") {
                if (!parse_uint(v, &u)) return cli_error(kConversion, "Could not convert: " + o + " = " + v);
                a->min_abundance = u;
            } else if (o == "-t" || o == "--threads") {
                if (!parse_int(v, &si)) return cli_error(kConversion, "Could not convert: " + o + " = " + v);
                if (si < 3 || si > 64) return cli_error(kValidation, o + ": Value " + v + " not in range 3 to 64");
                a->threads = (int)si;
            } else if (o == "-o" || o == "--output-file") {
                a->output = v;
            } else if (o == "-f" || o == "--bfilter-fpr") {
                if (!parse_double(v, &d)) return cli_error(kConversion, "Could not convert: " + o + " = " + v);
                if (!(d >= 0.001 && d <= 0.999))
                    return cli_error(kValidation, o + ": Value " + v + " not in range 0.001 to 0.999");
                a->fpr = d;
                a->fpr_set = true;
            } else if (o == "-s" || o == "--hash-tab-size") {
                if (!parse_uint(v, &u)) return cli_error(kConversion, "Could not convert: " + o + " = " + v);
                a->slots = u;
                a->have_s = true;
            } else if (o == "-u" || o == "--unq-kmers") {
                if (!parse_uint(v, &u)) return cli_error(kConversion, "Could not convert: " + o + " = " + v);
                a->unique = u;
                a->have_u = true;
            } else if (o == "--gunzip-to") {
                a->gunzip_to = v;
            } else if (o == "--device") {
                if (!parse_int(v, &si) || si < 0) return cli_error(kConversion, "Could not convert: " + o + " = " + v);
                a->device = (int)si;
            } else if (o == "--table-sizing") {
                if (v == "auto") a->table_sizing = 0;
                else if (v == "s") a->table_sizing = 1;
                else if (v == "estimate") a->table_sizing = 2;
                else return cli_error(kValidation, o + ": Value " + v + " not in {auto, s, estimate}");
            } else if (o == "--readers") {
                if (!parse_int(v, &si) || si < 1 || si > 16) return cli_error(kConversion, "Could not convert: " + o + " = " + v);
                a->readers = (unsigned)si;
            } else {
                return cli_error(kExtras, "The following argument was not expected: " + o);
            }
            continue;
        }
        pos.push_back(o);
    }
    if (pos.size() > 2) return cli_error(kExtras, "The following arguments were not expected: " + pos[2]);
    if (pos.size() < 1) return cli_error(kRequired, "INPUT is required");
    if (pos.size() < 2) return cli_error(kRequired, "KLEN is required");
    a->input = pos[0];
    struct stat st;
    if (stat(a->input.c_str(), &st) != 0 || S_ISDIR(st.st_mode))
        return cli_error(kValidation, "INPUT: File does not exist: " + a->input);
    if (!parse_int(pos[1], &a->k)) return cli_error(kConversion, "Could not convert: KLEN = " + pos[1]);
    if (a->k <= 0) return cli_error(kValidation, "KLEN: Value " + pos[1] + " not in range 0 to inf");
    if (a->have_s == a->have_u)
        return cli_error(kRequired, "[Option Group: dummy group2] Exactly 1 option from [-s,--hash-tab-size,-u,--unq-kmers] is required");
    if (a->use_bf && !a->have_u) return cli_error(kRequires, "--use-bfilter requires --unq-kmers");
    if (a->have_u && !a->use_bf) return cli_error(kRequires, "--unq-kmers requires --use-bfilter");
    if (a->fpr_set && !a->use_bf) return cli_error(kRequires, "--bfilter-fpr requires --use-bfilter");
    return -1;
}

std::string ext_of(const std::string& p) {  // std::filesystem::path::extension()
    size_t slash = p.find_last_of('/');
    std::string fn = slash == std::string::npos ? p : p.substr(slash + 1);
    size_t dot = fn.find_last_of('.');
    if (dot == std::string::npos || dot == 0 || fn == "..") return "";
    return fn.substr(dot);
}
std::string stem_of(const std::string& p) {
    size_t slash = p.find_last_of('/');
    std::string fn = slash == std::string::npos ? p : p.substr(slash + 1);
    size_t dot = fn.find_last_of('.');
    if (dot == std::string::npos || dot == 0) return fn;
    return fn.substr(0, dot);
}
std::string filename_of(const std::string& p) {
    size_t slash = p.find_last_of('/');
    return slash == std::string::npos ? p : p.substr(slash + 1);
}

// The input image in HBM: slices of the file (pread, fd >= 0) or of a host buffer
// (decompressed gzip) are copied by `readers` workers, each through two pinned slices and
// its own stream, so reading, H2D and the next read overlap.  prepare() allocates the image,
// the pinned slices, streams and events before the timed passes (as the reference allocates its
// table before its timer, parallel_parser.hpp:1230-1299): page-locking the slices was most of
// the upload's time.  run() then only reads and copies.  prepare() returns
// false (the caller stages host chunks instead) when the image does not fit comfortably in HBM.
struct Upload {
    uint8_t* d = nullptr;
    uint64_t size = 0, slice = 0, nslices = 0;
    struct Reader {
        hipStream_t st = nullptr;
        uint8_t* buf[2] = {nullptr, nullptr};
        hipEvent_t done[2] = {nullptr, nullptr};
    };
    std::vector<Reader> rd;
    // one reader: an event per slice and the slices issued so far (in file order), so that the
    // counting pass of a prefix can start while the rest uploads (wait_prefix)
    std::vector<hipEvent_t> sev;
    uint64_t issued = 0;
    bool failed = false;
    std::mutex mu;
    std::condition_variable cv;

    bool prepare(uint64_t sz, int device, unsigned readers) {
        size = sz;
        if (size == 0 || hipSetDevice(device) != hipSuccess) return false;
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess || size > fr / 4) return false;  // room for the passes
        if (hipMalloc(&d, size) != hipSuccess) {
            d = nullptr;
            return false;
        }
        slice = 8ull << 20;
        nslices = (size + slice - 1) / slice;
        readers = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(readers, nslices));
        // a slice per buffer no larger than the image: small inputs pin little
        const uint64_t bsz = std::min(slice, size);
        rd.resize(readers);
        if (readers == 1) {
            sev.assign(nslices, nullptr);
            for (auto& e : sev)
                if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail();
        }
        for (auto& r : rd) {
            if (hipStreamCreateWithFlags(&r.st, hipStreamNonBlocking) != hipSuccess) return fail();
            for (int b = 0; b < 2; b++)
                if (hipHostMalloc(&r.buf[b], bsz, hipHostMallocDefault) != hipSuccess ||
                    hipEventCreateWithFlags(&r.done[b], hipEventDisableTiming) != hipSuccess)
                    return fail();
        }
        return true;
    }
    bool release() {
        for (auto& e : sev)
            if (e) (void)hipEventDestroy(e);
        sev.clear();
        for (auto& r : rd) {
            for (int b = 0; b < 2; b++) {
                if (r.buf[b]) (void)hipHostFree(r.buf[b]);
                if (r.done[b]) (void)hipEventDestroy(r.done[b]);
                r.buf[b] = nullptr;
                r.done[b] = nullptr;
            }
            if (r.st) (void)hipStreamDestroy(r.st);
            r.st = nullptr;
        }
        rd.clear();
        return false;
    }
    void free_image() {
        if (d) (void)hipFree(d);
        d = nullptr;
    }
    bool fail() {
        release();
        free_image();
        return false;
    }
    // waits until the first `bytes` of the image are in HBM; false if the upload failed
    bool wait_prefix(uint64_t bytes) {
        const uint64_t need = std::min(nslices, (bytes + slice - 1) / slice);
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return failed || issued >= need; });
        if (failed) return false;
        lk.unlock();
        return need == 0 || hipEventSynchronize(sev[need - 1]) == hipSuccess;
    }
    // the image's bytes into d; false on a read or copy error (d is then freed unless keep_image:
    // a caller counting a prefix meanwhile frees it)
    bool run(int fd, const uint8_t* host, bool keep_image = false) {
        std::atomic<uint64_t> next{0};
        std::atomic<bool> bad{false};
        auto worker = [&](Reader& r) {
            bool ok = true, used[2] = {false, false};
            for (int b = 0; ok && !bad;) {
                const uint64_t i = next.fetch_add(1);
                if (i >= nslices) break;
                const uint64_t off = i * slice, len = std::min(slice, size - off);
                if (used[b] && hipEventSynchronize(r.done[b]) != hipSuccess) { ok = false; break; }
                if (fd >= 0) {
                    uint64_t got = 0;
                    while (got < len) {
                        const ssize_t n = pread(fd, r.buf[b] + got, len - got, (off_t)(off + got));
                        if (n <= 0) { ok = false; break; }
                        got += (uint64_t)n;
                    }
                } else {
                    std::memcpy(r.buf[b], host + off, len);
                }
                ok = ok && hipMemcpyAsync(d + off, r.buf[b], len, hipMemcpyHostToDevice, r.st) == hipSuccess &&
                     hipEventRecord(r.done[b], r.st) == hipSuccess;
                if (ok && !sev.empty()) {
                    ok = hipEventRecord(sev[i], r.st) == hipSuccess;
                    std::lock_guard<std::mutex> lk(mu);
                    issued = i + 1;
                    cv.notify_all();
                }
                used[b] = true;
                b ^= 1;
            }
            if (hipStreamSynchronize(r.st) != hipSuccess) ok = false;
            if (!ok) bad = true;
        };
        std::vector<std::thread> pool;
        for (size_t t = 1; t < rd.size(); t++) pool.emplace_back(worker, std::ref(rd[t]));
        worker(rd[0]);
        for (auto& t : pool) t.join();
        if (bad) {
            std::lock_guard<std::mutex> lk(mu);
            failed = true;
            cv.notify_all();
        }
        if (!bad) release();  // (after a failure a waiter may still hold a slice event)
        if (bad && !keep_image) free_image();
        return !bad;
    }
};

}  // namespace

int main(int argc, char** argv) {
    Args a;
    int prc = parse(argc, argv, &a);
    if (prc >= 0) return prc;

    // ---- format detection (main.cpp:19-68)
    int fd = open(a.input.c_str(), O_RDONLY);
    if (fd < 0) { std::cerr << "cannot open " << a.input << "\n"; return 1; }
    struct stat st;
    fstat(fd, &st);
    const uint64_t fsize = (uint64_t)st.st_size;
    unsigned char magic[2] = {0, 0};
    if (fsize >= 2) { ssize_t r = pread(fd, magic, 2, 0); (void)r; }
    const bool gz = magic[0] == 0x1f && magic[1] == 0x8b;
    std::string ext_path = a.input;
    if (gz) {
        while (ext_of(ext_path) == ".gz") ext_path = ext_path.substr(0, ext_path.size() - 3);
    }
    const std::string ext = ext_of(ext_path);

    // ---- load the image (mmap, or a full gunzip).  The reference's IO thread reads (and inflates)
    // the file and cuts its chunks inside its timers (parallel_parser.hpp:1230-1299,1544-1550): the
    // time of both is added to the first timer line below
    using clk = std::chrono::high_resolution_clock;
    const auto t_in0 = clk::now();
    const uint8_t* image = nullptr;
    uint64_t isize = 0;
    std::vector<uint8_t> gzbuf;
    void* map = nullptr;
    bool bgzf = false;
    if (gz) {  // BGZF: members inflated in parallel
        void* zm = mmap(nullptr, fsize, PROT_READ, MAP_PRIVATE, fd, 0);
        if (zm != MAP_FAILED) {
            const unsigned hw = std::thread::hardware_concurrency();
            bool bad = false;
            bgzf = gunzip_bgzf((const uint8_t*)zm, fsize, (int)std::min(16u, hw ? hw : 1u), &gzbuf, &bad);
            munmap(zm, fsize);
            if (bgzf && bad) {
                std::cerr << "gzip input " << a.input << " is corrupt or truncated: a BGZF member does not inflate"
                          << std::endl;
                return 1;
            }
        }
    }
    if (gz && !bgzf) {
        gzFile g = gzdopen(dup(fd), "r");
        if (!g) { std::cerr << "cannot open " << a.input << " as gzip\n"; return 1; }
        gzbuffer(g, 1 << 20);
        std::vector<uint8_t> tmp(1 << 22);
        int n;
        while ((n = gzread(g, tmp.data(), (unsigned)tmp.size())) > 0) gzbuf.insert(gzbuf.end(), tmp.begin(), tmp.begin() + n);
        int zerr = Z_OK;
        const char* msg = gzerror(g, &zerr);
        // corrupt or truncated stream (zlib reports a cut stream as Z_BUF_ERROR after
        // returning what it decoded): fail instead of counting a prefix
        if (n < 0 || (zerr != Z_OK && zerr != Z_STREAM_END)) {
            std::cerr << "gzip input " << a.input << " is corrupt or truncated: " << (msg ? msg : "") << std::endl;
            gzclose(g);
            return 1;
        }
        gzclose(g);
    }
    if (gz) {
        image = gzbuf.data();
        isize = gzbuf.size();
    } else if (fsize) {
        map = mmap(nullptr, fsize, PROT_READ, MAP_PRIVATE, fd, 0);
        if (map == MAP_FAILED) { std::cerr << "mmap failed\n"; return 1; }
        madvise(map, fsize, MADV_SEQUENTIAL);
        image = (const uint8_t*)map;
        isize = fsize;
    }
    if (!a.gunzip_to.empty()) {  // test hook (tests/test_host.py): the decompressed bytes, no GPU work
        FILE* f = std::fopen(a.gunzip_to.c_str(), "wb");
        if (!f || (isize && std::fwrite(image, 1, isize, f) != isize)) { std::cerr << "cannot write " << a.gunzip_to << "\n"; return 1; }
        std::fclose(f);
        std::cout << "gunzip: " << isize << " bytes" << (bgzf ? " (BGZF, parallel)" : "") << std::endl;
        return 0;
    }
    const unsigned char sym = isize ? image[0] : 0;
    int fmt;
    bool ill = false;
    if (ext == ".fasta" || ext == ".fa") { fmt = KC_FMT_FASTA; ill = sym != '>'; }
    else if (ext == ".fastq" || ext == ".fq") { fmt = KC_FMT_FASTQ; ill = sym != '@'; }
    else { fmt = KC_FMT_PLAIN; ill = !(sym && std::strchr("actgACGT", sym)); }
    if (ill) {
        std::cerr << "Input file " << a.input << " is ill-formed" << std::endl;
        return 1;
    }
    if (a.output.empty()) a.output = stem_of(a.input) + ".kaarme_counts";

    std::cout << "Running settings: " << std::endl;
    std::cout << "  input file:               " << filename_of(a.input) << std::endl;
    std::cout << "  input format:             " << (fmt == KC_FMT_FASTA ? "FASTA" : fmt == KC_FMT_FASTQ ? "FASTQ" : "ONE-STR-PER-LINE") << std::endl;
    std::cout << "  gzip compressed:          " << (gz ? "yes" : "no") << std::endl;
    std::cout << "  k-mer length:             " << a.k << std::endl;
    std::cout << "  min. abundance threshold: " << a.min_abundance << std::endl;
    std::cout << "  hash table type:          " << (a.mode == 0 ? "plain" : "kaarme") << std::endl;
    std::cout << "  using bloom filers:       " << (a.use_bf ? "yes" : "no") << std::endl;
    if (a.use_bf) {
        std::cout << "    est. unique k-mers:     " << a.unique << std::endl;
        std::cout << "    false positive rate:    " << a.fpr << std::endl;
    } else {
        std::cout << "    est. hash table size:   " << a.slots << std::endl;
    }
    std::cout << "  working threads:          " << a.threads << std::endl;
    std::cout << "  output file:              " << a.output << std::endl;
    std::cout << "  device:                   MI355X (HIP device " << a.device << ")" << std::endl;

    if (a.k > KC_MAX_K) {  // fifteen 64-bit key words (include/kc_api.h); INTEGRATION.md "Differences"
        std::cerr << "k-mer length above " << KC_MAX_K << " is not supported by this build" << std::endl;
        return 1;
    }

    const auto t_in1 = clk::now();  // (the input's bytes are in host memory: mapped, or inflated)
    kc_chunk* chunks = nullptr;
    uint64_t nch = 0;
    if (kc_plan_chunks(image, isize, (int)a.k, 0, fmt, &chunks, &nch) != KC_OK) {
        std::cerr << "chunk planning failed" << std::endl;
        return 1;
    }
    const auto t_in2 = clk::now();
    // (an uncompressed file is mapped lazily: its bytes are read by the timed upload, so only the
    // planning counts; a gzip file is inflated here, which the reference does inside its timer)
    const long long prep_us =
        (long long)std::chrono::duration_cast<std::chrono::microseconds>(t_in2 - (gz ? t_in0 : t_in1)).count();

    kc_config cfg;
    std::memset(&cfg, 0, sizeof(cfg));
    cfg.k = (int)a.k;
    cfg.mode = a.mode;
    cfg.bf_enable = a.use_bf;
    cfg.device = a.device;
    cfg.table_slots = a.slots;
    cfg.est_unique = a.unique;
    cfg.fpr = a.fpr;
    cfg.min_abundance = a.min_abundance;
    {   // a small input gets a stage of its own size (one batch, little pinned memory);
        // larger ones the library's default (sized from free HBM)
        uint64_t staged = 4096;
        for (uint64_t i = 0; i < nch; i++) staged += (chunks[i].len + 4095) / 4096 * 4096;
        if (staged <= (256ull << 20)) cfg.batch_bytes = staged;
    }
    kc_ctx* ctx = nullptr;
    if (kc_create(&cfg, &ctx) != KC_OK) {
        std::cerr << "kc_create: " << kc_last_error(nullptr) << std::endl;
        return 1;
    }
    auto die = [&](const char* what) {
        std::cerr << what << ": " << kc_last_error(ctx) << std::endl;
        kc_destroy(ctx);
        std::exit(1);
    };
    // The image goes to HBM once (--host-chunks: stage host chunks instead): both passes
    // then read it in place, and a Bloom job counts from the Bloom pass's partitions
    // (kc_api.h, partition reuse).  Its read is timed with the pass that needs it first,
    // as the reference's reader thread is.  (One reader by default: the C2 sample's timed build
    // 25-28 ms after the warm-up below, against 32-35 ms with two and more with four;
    // profiles/r04_cli_probe_{phases,warmup}.txt)
    const bool host_path = a.host_chunks;
    Upload up;
    const bool staged = !host_path && up.prepare(isize, a.device, a.readers);  // (untimed setup)
    if (staged && !a.no_warmup) {
        // (untimed setup, as the reference's table allocation is) the GPU runtime's one-time
        // work -- loading the counting kernels' code, first launches -- on a one-read input: a
        // -s job on its own context, then kc_reset; a -b job on a small context of its own (a
        // Bloom pass, finalize and the gated pass load the Bloom kernels; the job's context keeps
        // its create-time fine geometry), so the timed passes start on a warm device
        static const char kWarm[] = ">w\nACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGT\n";
        // the read through the partitioned levels the timed pass takes (a read this short
        // would take the direct path), unless the caller forces a path
        const bool force = std::getenv("KC_INSERT_PATH") == nullptr;
        if (force) setenv("KC_INSERT_PATH", "partitioned", 1);
        uint8_t* dw = nullptr;
        const kc_chunk wc{0, sizeof(kWarm) - 1, 0, 0};
        if (hipMalloc(&dw, sizeof(kWarm)) == hipSuccess) {
            if (hipMemcpy(dw, kWarm, sizeof(kWarm) - 1, hipMemcpyHostToDevice) == hipSuccess) {
                if (!a.use_bf) {
                    if (kc_count_device(ctx, dw, &wc, 1, KC_FMT_FASTA, nullptr) == KC_OK) (void)kc_sync(ctx);
                } else {
                    kc_config w = cfg;
                    w.est_unique = 1000;
                    w.batch_bytes = 1 << 20;
                    kc_ctx* wctx = nullptr;
                    uint64_t nis = 0;
                    if (kc_create(&w, &wctx) == KC_OK && kc_bloom_device(wctx, dw, &wc, 1, KC_FMT_FASTA, nullptr) == KC_OK &&
                        kc_bloom_finalize(wctx, &nis) == KC_OK &&
                        kc_count_device(wctx, dw, &wc, 1, KC_FMT_FASTA, nullptr) == KC_OK)
                        (void)kc_sync(wctx);
                    kc_destroy(wctx);
                }
            }
            (void)hipFree(dw);
        }
        if (force) unsetenv("KC_INSERT_PATH");
        if (!a.use_bf && kc_reset(ctx) != KC_OK) die("reset after warm-up");
    }
    // A -s whose table would take a large share of HBM is sized from the input's distinct estimate
    // inside the timer (below).  Its -s table, allocated by kc_create, is given back first (untimed
    // setup, as the reference's table allocation): beside C5's 192 GB -s table the 10 GB upload
    // crawled at 1.7 GB/s (5.8 s; 0.35 s beside a 96 GB table, profiles/r06_cli_c5_phases.txt)
    const int kw = (int)(a.k / 32 + 1);
    const double s_table_bytes = 1.25 * (double)a.slots / (double)(16 / (kw + 1)) * 128.0;
    const bool want_est = a.table_sizing == 2 || (a.table_sizing == 0 && s_table_bytes > (double)(16ull << 30) && nch > 1);
    bool s_table_dropped = false;
    if (staged && !a.use_bf && want_est) s_table_dropped = kc_size_table(ctx, 1u << 20) == KC_OK;
    uint8_t* d_img = nullptr;
    bool loaded = false;
    auto load = [&]() {
        if (staged && !loaded) {
            loaded = true;
            if (up.run(gz ? -1 : fd, image)) d_img = up.d;
        }
    };
    uint64_t bf_new_in_second = 0;
    if (a.use_bf) {
        std::cout << "Starting parallel bloom filtering\n";
        auto t0 = clk::now();
        load();
        if (d_img) {
            if (kc_bloom_device(ctx, d_img, chunks, nch, fmt, nullptr) != KC_OK) die("bloom pass");
        } else {
            for (uint64_t i = 0; i < nch; i++)
                if (kc_bloom_chunk(ctx, image + chunks[i].off, chunks[i].len, fmt, chunks[i].broken_header) != KC_OK)
                    die("bloom pass");
        }
        uint64_t nis = 0;
        if (kc_bloom_finalize(ctx, &nis) != KC_OK) die("bloom finalize");
        bf_new_in_second = nis;
        auto t1 = clk::now();
        std::cout << "New k-mers in second bloom filter " << nis << "\n";
        std::cout << "Time used to bloom filter k-mers: "
                  << std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count() + prep_us
                  << " microseconds\n";
    }
    std::cout << "Starting " << (a.mode == 0 ? "atomic flag basic" : "atomic variable pointer") << " hash table\n";
    const bool dbg = a.phases;  // phase times on stderr
    auto us = [](clk::time_point x, clk::time_point y) {
        return (long long)std::chrono::duration_cast<std::chrono::microseconds>(y - x).count();
    };
    auto t0 = clk::now();
    // A -s whose table would take a large share of HBM (C4's -s 2.6e9 asks for 83 GB at 25 %
    // headroom; its 1.0 G distinct k-mers need 35 GB) is sized from the whole input's distinct
    // estimate instead (kc_estimate_distinct_device + kc_size_table, inside the timer; -s stays
    // the reference capacity for --strict-capacity), as bench.py's C4 / C5 lines are.  A table
    // that still fills up (an estimate far below the truth) is counted again at -s.
    bool est_sized = false;
    if (staged && !loaded && !a.use_bf && want_est) {
        load();
        double est = 0;
        if (d_img && kc_estimate_distinct_device(ctx, d_img, chunks, nch, fmt, nullptr, &est) == KC_OK) {
            const double want = 1.1 * est + (double)(1 << 20);
            if ((want < 0.8 * (double)a.slots || a.table_sizing == 2) && kc_size_table(ctx, (uint64_t)want) == KC_OK) {
                est_sized = true;
                if (dbg) std::cerr << "cli: table sized from the distinct estimate " << (uint64_t)est << "\n";
            }
        }
    }
    if (s_table_dropped && !est_sized && kc_size_table(ctx, 0) != KC_OK) die("sizing the -s table");
    // A large -s job counts the image's first half while the second half uploads (two counting
    // passes into one table: the second sweeps it once more, ~1.5 ms for C2's, against ~8 ms of
    // the upload hidden); a Bloom job's counting pass follows the Bloom pass, which read it all
    uint64_t split = 0;
    if (staged && !loaded && !a.use_bf && isize >= (512ull << 20) && up.sev.size() && nch > 1) {
        while (split < nch && chunks[split].off + chunks[split].len < isize / 2) split++;
        split = std::min<uint64_t>(split + 1, nch - 1);
    }
    if (split) {
        loaded = true;
        bool up_ok = false;
        std::thread reader([&] { up_ok = up.run(gz ? -1 : fd, image, true); });
        const uint64_t pre_end = chunks[split - 1].off + chunks[split - 1].len + 4096;
        const bool pre_ok = up.wait_prefix(std::min(isize, pre_end));
        const int rc1 = pre_ok ? kc_count_device(ctx, up.d, chunks, split, fmt, nullptr) : KC_OK;
        reader.join();
        up.release();
        if (!pre_ok || !up_ok) {
            up.free_image();
            die("uploading the input");
        }
        if (rc1 != KC_OK) die("counting pass");
        d_img = up.d;
        if (kc_count_device(ctx, d_img, chunks + split, nch - split, fmt, nullptr) != KC_OK) die("counting pass");
        if (dbg) std::cerr << "cli: overlapped upload, counting passes of " << split << " + " << nch - split << " chunks\n";
    } else {
    load();
    auto tl = clk::now();
    if (d_img) {
        if (kc_count_device(ctx, d_img, chunks, nch, fmt, nullptr) != KC_OK) die("counting pass");
        if (dbg) {
            auto tc = clk::now();
            (void)kc_sync(ctx);
            std::cerr << "cli: load " << us(t0, tl) << " us, count call " << us(tl, tc) << " us, its work "
                      << us(tc, clk::now()) << " us\n";
        }
    } else {
        for (uint64_t i = 0; i < nch; i++)
            if (kc_count_chunk(ctx, image + chunks[i].off, chunks[i].len, fmt, chunks[i].broken_header) != KC_OK)
                die("counting pass");
    }
    }
    kc_stats stt;
    int frc = kc_finish(ctx, &stt);
    if (frc == KC_ERR_TABLE_FULL && est_sized) {  // the estimate was too low: the -s table, counted again
        std::cerr << "cli: the estimate-sized table filled up; counting again into the -s table\n";
        if (kc_reset(ctx) != KC_OK || kc_size_table(ctx, 0) != KC_OK ||
            kc_count_device(ctx, d_img, chunks, nch, fmt, nullptr) != KC_OK)
            die("counting pass");
        est_sized = false;
        frc = kc_finish(ctx, &stt);
    }
    if (frc != KC_OK) {
        std::cout << "Hash table is full... Cannot handle this yet\n";
        die("counting pass");
    }
    auto t1 = clk::now();
    // the reference prints its table size, next_prime3mod4(-s or 2 * new_in_second)
    // (functions_math.cpp:90); the device table keeps 25 % headroom over it
    const uint64_t ref_slots = kc_table_size_reference(a.use_bf ? 2 * bf_new_in_second : a.slots);
    std::cout << "Hash table size is: " << ref_slots << "\n";
    if (a.min_abundance > 0 && a.digest_only) {
        // --digest-only (extension): the output's order-independent digest (kc_output_digest: lines,
        // sum of T(c), sum and XOR of XXH64 per line) instead of the file -- C4's 60 GB of text
        kc_digest dg;
        if (kc_output_digest(ctx, &dg) != KC_OK) die("output digest");
        char buf[200];
        std::snprintf(buf, sizeof buf, "{\"lines\": %llu, \"count_sum\": %llu, \"hash_sum\": \"%016llx\", \"hash_xor\": \"%016llx\"}",
                      (unsigned long long)dg.lines, (unsigned long long)dg.count_sum, (unsigned long long)dg.hash_sum,
                      (unsigned long long)dg.hash_xor);
        std::cout << "Output digest: " << buf << "\n";
    } else if (a.min_abundance > 0) {
        std::cout << "Start writing k-mers in a file\n";
        if (kc_write(ctx, a.output.c_str()) != KC_OK) die("writing k-mers");
    }
    auto t2 = clk::now();
    std::cout << "Time used to build hash table: "
              << std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count() + (a.use_bf ? 0 : prep_us)
              << " microseconds\n";
    std::cout << "Input read and chunked in " << prep_us << " microseconds (included in the first timer line)\n";
    if (est_sized)
        std::cout << "Device table sized from the distinct estimate (-s " << a.slots
                  << " stays the reference capacity)\n";
    std::cout << "Time used to write k-mers in a file: "
              << std::chrono::duration_cast<std::chrono::microseconds>(t2 - t1).count() << " microseconds\n";
    std::cout << "Processed k-mers: " << stt.windows << " (inserted " << stt.inserted << ")\n";
    std::cout << "Main array slots used " << stt.distinct << " / " << ref_slots << "\n";
    std::cout << "Device table capacity: " << stt.table_slots << " slots\n";
    std::cout << "Input path: " << (d_img ? "device image" : "host chunks")
              << (stt.reused_passes ? " (counting pass from the Bloom pass's partitions)" : "") << "\n";
    kc_destroy(ctx);
    up.release();
    up.free_image();
    kc_free(chunks);
    if (map) munmap(map, fsize);
    close(fd);
    return 0;
}
