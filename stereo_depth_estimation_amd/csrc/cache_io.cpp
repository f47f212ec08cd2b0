// Native host readers for the data path: the reference's sample cache and its PNG frames.
// Sample cache (reference dataset.py:86-105 load_cached_sample, cache.py:50-112):
// one np.savez file per pair, a zip of left.npy / right.npy (uint8 HWC) and disparity.npy (f16 HW): stored members
// (np.savez, the default) or raw-deflate members (np.savez_compressed, the reference's `cache.py --compress`).
// A batch of files is read by a pool of threads straight into the caller's (pinned) host buffers, so the data path
// needs no worker processes, no pickling and no second pinning copy (tools/loader_bench.py: the torch DataLoader
// path tops out near 3-4k pairs/s on the box's 16 cores).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

uint16_t rd16(const unsigned char* p) { return (uint16_t)(p[0] | p[1] << 8); }
uint32_t rd32(const unsigned char* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
uint64_t rd64(const unsigned char* p) { return (uint64_t)rd32(p) | (uint64_t)rd32(p + 4) << 32; }

bool read_file(const char* path, std::vector<unsigned char>& buf, std::string& why) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) {
        why = "cannot open";
        return false;
    }
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        why = "cannot stat";
        return false;
    }
    buf.resize((size_t)st.st_size);
    size_t got = 0;
    while (got < buf.size()) {
        const ssize_t r = read(fd, buf.data() + got, buf.size() - got);
        if (r <= 0) break;
        got += (size_t)r;
    }
    close(fd);
    if (got != buf.size()) {
        why = "short read";
        return false;
    }
    return true;
}

// the .npy payload of one stored zip member, checked against dtype descr and the expected shape text
bool npy_payload(const unsigned char* p, size_t n, const char* descr, const std::string& shape, size_t bytes,
                 const unsigned char** data, std::string& why) {
    if (n < 10 || memcmp(p, "\x93NUMPY", 6) != 0) {
        why = "not an .npy member";
        return false;
    }
    const int major = p[6];
    const size_t hl = major == 1 ? rd16(p + 8) : rd32(p + 8);
    const size_t off = major == 1 ? 10 : 12;
    if (off + hl > n) {
        why = "truncated .npy header";
        return false;
    }
    const std::string hdr((const char*)p + off, hl);
    if (hdr.find(std::string("'descr': '") + descr + "'") == std::string::npos ||
        hdr.find("'fortran_order': False") == std::string::npos ||
        hdr.find("'shape': " + shape) == std::string::npos) {
        why = "dtype/shape mismatch (" + hdr.substr(0, hdr.find('}') + 1) + ")";
        return false;
    }
    if (off + hl + bytes > n) {
        why = "truncated .npy data";
        return false;
    }
    *data = p + off + hl;
    return true;
}

// a raw-deflate zip member (method 8) inflated into `out` (exactly usize bytes)
bool inflate_member(const unsigned char* src, size_t csize, size_t usize, std::vector<unsigned char>& out,
                    std::string& why) {
    out.resize(usize);
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, -MAX_WBITS) != Z_OK) {
        why = "inflateInit2 failed";
        return false;
    }
    zs.next_in = const_cast<unsigned char*>(src);
    zs.avail_in = (uInt)csize;
    zs.next_out = out.data();
    zs.avail_out = (uInt)usize;
    const int rc = inflate(&zs, Z_FINISH);
    const size_t got = zs.total_out;
    inflateEnd(&zs);
    if (rc != Z_STREAM_END || got != usize) {
        why = "corrupt deflate member";
        return false;
    }
    return true;
}

// walks the zip's local headers (sizes in the header or its zip64 extra field); members stored (np.savez) or
// deflated (np.savez_compressed), inflated into `scratch`
bool parse_npz(const std::vector<unsigned char>& f, int H, int W, unsigned char* left, unsigned char* right,
               uint16_t* disp, std::vector<unsigned char>& scratch, std::string& why) {
    const std::string s3 = "(" + std::to_string(H) + ", " + std::to_string(W) + ", 3)";
    const std::string s2 = "(" + std::to_string(H) + ", " + std::to_string(W) + ")";
    const size_t rgb = (size_t)H * W * 3, dbytes = (size_t)H * W * 2;
    int found = 0;
    size_t pos = 0;
    while (pos + 30 <= f.size() && rd32(&f[pos]) == 0x04034b50u) {
        const unsigned char* h = &f[pos];
        const uint16_t flags = rd16(h + 6), method = rd16(h + 8), nlen = rd16(h + 26), xlen = rd16(h + 28);
        uint64_t csize = rd32(h + 18), usize = rd32(h + 22);
        if (pos + 30 + nlen + xlen > f.size()) break;
        const std::string name((const char*)h + 30, nlen);
        if (csize == 0xffffffffu || usize == 0xffffffffu) {  // zip64 extra field: usize, csize
            const unsigned char* x = h + 30 + nlen;
            for (size_t k = 0; k + 4 <= xlen;) {
                const uint16_t id = rd16(x + k), sz = rd16(x + k + 2);
                if (id == 1 && sz >= 16) {
                    usize = rd64(x + k + 4);
                    csize = rd64(x + k + 12);
                }
                k += 4 + sz;
            }
        }
        if ((method != 0 && method != 8) || (flags & 8) || (method == 0 && csize != usize)) {
            why = "member " + name + " uses an unsupported zip method or is streamed (not np.savez output)";
            return false;
        }
        const size_t data = pos + 30 + nlen + xlen;
        if (data + csize > f.size()) break;
        const bool wanted = name == "left.npy" || name == "right.npy" || name == "disparity.npy";
        const unsigned char* mem = &f[data];
        if (wanted && method == 8) {
            if (usize > ((size_t)1 << 32) || !inflate_member(mem, csize, usize, scratch, why)) {
                why = name + ": " + (why.empty() ? "member too large" : why);
                return false;
            }
            mem = scratch.data();
        }
        const unsigned char* src = nullptr;
        if (name == "left.npy" || name == "right.npy") {
            if (!npy_payload(mem, usize, "|u1", s3, rgb, &src, why)) {
                why = name + ": " + why;
                return false;
            }
            memcpy(name[0] == 'l' ? left : right, src, rgb);
            found |= name[0] == 'l' ? 1 : 2;
        } else if (name == "disparity.npy") {
            if (!npy_payload(mem, usize, "<f2", s2, dbytes, &src, why)) {
                why = name + ": " + why;
                return false;
            }
            memcpy(disp, src, dbytes);
            found |= 4;
        }
        pos = data + csize;
    }
    if (found != 7) {
        why = "missing left/right/disparity member";
        return false;
    }
    return true;
}

}  // namespace

extern "C" int sd_read_cache_batch(const char* const* paths, int n, int H, int W, uint8_t* left, uint8_t* right,
                                   uint16_t* disparity, int threads, char* err, int errlen) {
    if (!paths || n < 0 || H <= 0 || W <= 0 || !left || !right || !disparity) {
        if (err && errlen > 0) snprintf(err, (size_t)errlen, "sd_read_cache_batch: bad args");
        return -1;
    }
    if (threads < 1) threads = 1;
    if (threads > n) threads = n > 0 ? n : 1;
    const size_t rgb = (size_t)H * W * 3, hw = (size_t)H * W;
    std::atomic<int> next{0}, first_bad{n};
    std::mutex mu;
    std::string bad_why;
    auto work = [&]() {
        std::vector<unsigned char> buf, scratch;
        std::string why;
        for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) {
            bool ok = paths[i] && read_file(paths[i], buf, why);
            if (ok) ok = parse_npz(buf, H, W, left + i * rgb, right + i * rgb, disparity + i * hw, scratch, why);
            if (!ok) {
                std::lock_guard<std::mutex> g(mu);
                if (i < first_bad.load()) {
                    first_bad.store(i);
                    bad_why = why;
                }
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    const int bad = first_bad.load();
    if (bad < n) {
        if (err && errlen > 0)
            snprintf(err, (size_t)errlen, "%s: %s", paths[bad] ? paths[bad] : "(null)", bad_why.c_str());
        return bad + 1;
    }
    return 0;
}

// ------------------------------------------------------------------ PNG frames (the un-cached source)
// FoundationStereo frames and the RGB24 disparity codec images (reference dataset.py:23-30,184-212) are 8-bit RGB
// or RGBA PNGs, not interlaced. Decoded here as PIL's Image.open(p).convert("RGB") returns them (alpha dropped);
// other PNG kinds report an error and the caller falls back to PIL.

namespace {

uint32_t be32(const unsigned char* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

bool png_header(const std::vector<unsigned char>& f, int& w, int& h, int& bpp, std::string& why) {
    static const unsigned char sig[8] = {0x89, 'P', 'N', 'G', 0x0d, 0x0a, 0x1a, 0x0a};
    if (f.size() < 33 || memcmp(f.data(), sig, 8) != 0 || memcmp(&f[12], "IHDR", 4) != 0) {
        why = "not a PNG";
        return false;
    }
    w = (int)be32(&f[16]);
    h = (int)be32(&f[20]);
    const int depth = f[24], color = f[25], interlace = f[28];
    if (depth != 8 || (color != 2 && color != 6) || interlace != 0 || f[26] != 0 || f[27] != 0) {
        why = "unsupported PNG kind (needs 8-bit RGB/RGBA, not interlaced)";
        return false;
    }
    bpp = color == 2 ? 3 : 4;
    return true;
}

unsigned char paeth(int a, int b, int c) {
    const int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
    return (unsigned char)(pa <= pb && pa <= pc ? a : (pb <= pc ? b : c));
}

bool decode_png(const std::vector<unsigned char>& f, int H, int W, unsigned char* out, std::vector<unsigned char>& z,
                std::vector<unsigned char>& raw, std::string& why) {
    int w = 0, h = 0, bpp = 0;
    if (!png_header(f, w, h, bpp, why)) return false;
    if (w != W || h != H) {
        why = "size " + std::to_string(h) + "x" + std::to_string(w) + " differs from the batch's";
        return false;
    }
    z.clear();
    for (size_t pos = 8; pos + 12 <= f.size();) {
        const uint32_t len = be32(&f[pos]);
        if (pos + 12 + (size_t)len > f.size()) break;
        const unsigned char* type = &f[pos + 4];
        if (memcmp(type, "IDAT", 4) == 0) z.insert(z.end(), f.begin() + pos + 8, f.begin() + pos + 8 + len);
        if (memcmp(type, "IEND", 4) == 0) break;
        pos += 12 + (size_t)len;
    }
    const size_t stride = (size_t)W * bpp;
    raw.resize((size_t)H * (stride + 1));
    uLongf got = (uLongf)raw.size();
    if (uncompress(raw.data(), &got, z.data(), (uLong)z.size()) != Z_OK || got != raw.size()) {
        why = "corrupt image data";
        return false;
    }
    for (int y = 0; y < H; ++y) {  // unfilter in place (filter byte, then the row)
        unsigned char* row = &raw[(size_t)y * (stride + 1) + 1];
        const unsigned char* up = y ? &raw[(size_t)(y - 1) * (stride + 1) + 1] : nullptr;
        const int ft = row[-1];
        for (size_t x = 0; x < stride; ++x) {
            const int a = x >= (size_t)bpp ? row[x - bpp] : 0, b = up ? up[x] : 0;
            const int c = (up && x >= (size_t)bpp) ? up[x - bpp] : 0;
            switch (ft) {
                case 0: break;
                case 1: row[x] = (unsigned char)(row[x] + a); break;
                case 2: row[x] = (unsigned char)(row[x] + b); break;
                case 3: row[x] = (unsigned char)(row[x] + ((a + b) >> 1)); break;
                case 4: row[x] = (unsigned char)(row[x] + paeth(a, b, c)); break;
                default: why = "bad filter type"; return false;
            }
        }
        unsigned char* o = out + (size_t)y * W * 3;
        if (bpp == 3) {
            memcpy(o, row, stride);
        } else {
            for (int x = 0; x < W; ++x) {
                o[3 * x] = row[4 * x];
                o[3 * x + 1] = row[4 * x + 1];
                o[3 * x + 2] = row[4 * x + 2];
            }
        }
    }
    return true;
}

}  // namespace

extern "C" int sd_png_size(const char* path, int* height, int* width) {
    std::vector<unsigned char> f;
    std::string why;
    int bpp = 0;
    if (!path || !height || !width || !read_file(path, f, why) || !png_header(f, *width, *height, bpp, why)) return -1;
    return 0;
}

extern "C" int sd_read_png_batch(const char* const* paths, int n, int H, int W, uint8_t* out, int threads, char* err,
                                 int errlen) {
    if (!paths || n < 0 || H <= 0 || W <= 0 || !out) {
        if (err && errlen > 0) snprintf(err, (size_t)errlen, "sd_read_png_batch: bad args");
        return -1;
    }
    if (threads < 1) threads = 1;
    if (threads > n) threads = n > 0 ? n : 1;
    std::atomic<int> next{0}, first_bad{n};
    std::mutex mu;
    std::string bad_why;
    auto work = [&]() {
        std::vector<unsigned char> buf, z, raw;
        std::string why;
        for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) {
            bool ok = paths[i] && read_file(paths[i], buf, why);
            if (ok) ok = decode_png(buf, H, W, out + (size_t)i * H * W * 3, z, raw, why);
            if (!ok) {
                std::lock_guard<std::mutex> g(mu);
                if (i < first_bad.load()) {
                    first_bad.store(i);
                    bad_why = why;
                }
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    const int bad = first_bad.load();
    if (bad < n) {
        if (err && errlen > 0)
            snprintf(err, (size_t)errlen, "%s: %s", paths[bad] ? paths[bad] : "(null)", bad_why.c_str());
        return bad + 1;
    }
    return 0;
}
