// Packed galaxy batches: host-side reader of the GDPACK01 file format.
//
// The reference feeds its models one galaxy at a time: Galaxy_Dataset.__getitem__
// (utils/utils_data.py:87-103) does three torch.load calls per galaxy (psf_{i}.pth, obs_{i}.pth,
// gt_{i}.pth) and computes alpha = obs.mean(); the test loader runs at batch size 1 (:135).  A batch of
// 4096 galaxies at 256^2 is 1 GiB of observations - 12k pickle loads - while the HIP engine deconvolves
// it in ~17 ms.  GDPACK01 stores a whole dataset as four contiguous fp32 sections (obs [n][H][W],
// psf [n][h][w], gt [n][H][W] (optional), alpha [n]) plus the dataset's info.json, so a batch is one
// contiguous byte range per section, read here by a pool of pread() threads straight into the
// caller's (pinned) host buffer; the H2D copy and its overlap with compute are the caller's
// (gdeconv/ingest.py: double-buffered pinned staging + a copy stream).
//
// Layout (little-endian): bytes [0, 8) "GDPACK01"; int64 n; int32 H, W, h, w, has_gt, reserved;
// int64 offset[5], bytes[5] for sections obs, psf, gt, alpha, info (UTF-8 JSON); each section starts
// on a 4096-byte boundary; the header occupies the first 4096 bytes.
#pragma once
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace gd {
namespace ingest {

constexpr char kMagic[8] = {'G', 'D', 'P', 'A', 'C', 'K', '0', '1'};
constexpr int kSections = 5;  // GD_PACK_OBS, _PSF, _GT, _ALPHA, _INFO

struct Header {
    char magic[8];
    int64_t n;
    int32_t H, W, h, w, has_gt, reserved;
    int64_t offset[kSections];
    int64_t bytes[kSections];
};
static_assert(sizeof(Header) == 8 + 8 + 6 * 4 + 2 * kSections * 8, "packed header layout");

struct Pack {
    int fd = -1;
    Header hd;
    int64_t file_bytes = 0;
    int64_t item_bytes(int sec) const {
        switch (sec) {
            case 0: case 2: return (int64_t)hd.H * hd.W * 4;
            case 1: return (int64_t)hd.h * hd.w * 4;
            case 3: return 4;
            default: return 1;
        }
    }
};

// Read [off, off + len) into dst with whole-range pread loops (short reads and EINTR retried).
inline bool pread_all(int fd, char* dst, int64_t off, int64_t len) {
    while (len > 0) {
        const ssize_t r = ::pread(fd, dst, (size_t)(len < (int64_t(1) << 30) ? len : (int64_t(1) << 30)), (off_t)off);
        if (r < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        if (r == 0) return false;  // truncated file
        dst += r;
        off += r;
        len -= r;
    }
    return true;
}

// Split `total` work items over up to `nthreads` threads (the calling thread takes a share).
template <typename F>
bool parallel_for(int64_t total, int nthreads, F&& f) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    if ((int64_t)nthreads > total) nthreads = total > 0 ? (int)total : 1;
    std::vector<char> ok(nthreads, 1);
    std::vector<std::thread> th;
    const int64_t per = (total + nthreads - 1) / nthreads;
    for (int t = 1; t < nthreads; ++t) {
        const int64_t b = t * per, e = b + per < total ? b + per : total;
        if (b >= e) break;
        th.emplace_back([&, t, b, e] { ok[t] = f(b, e) ? 1 : 0; });
    }
    ok[0] = f(0, per < total ? per : total) ? 1 : 0;
    for (auto& x : th) x.join();
    for (char c : ok)
        if (!c) return false;
    return true;
}

}  // namespace ingest
}  // namespace gd

extern "C" {

int gd_pack_open(const char* path, void** handle, long long* n, int* dims) {
    using namespace gd::ingest;
    if (!path || !handle) return fail(GD_ERR_ARG, "gd_pack_open: null argument");
    *handle = nullptr;
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return fail(GD_ERR_ARG, std::string("gd_pack_open: cannot open ") + path + ": " + std::strerror(errno));
    Pack* p = new Pack;
    p->fd = fd;
    struct stat sb;
    if (::fstat(fd, &sb) != 0 || !pread_all(fd, reinterpret_cast<char*>(&p->hd), 0, sizeof(Header)) ||
        std::memcmp(p->hd.magic, kMagic, 8) != 0) {
        ::close(fd);
        delete p;
        return fail(GD_ERR_ARG, std::string("gd_pack_open: ") + path + " is not a GDPACK01 file");
    }
    p->file_bytes = sb.st_size;
    const Header& h = p->hd;
    bool good = h.n >= 0 && h.H > 0 && h.W > 0 && h.h > 0 && h.w > 0;
    for (int s = 0; s < kSections && good; ++s) {
        if (s == 2 && !h.has_gt) continue;
        const int64_t need = s == 4 ? h.bytes[4] : h.n * p->item_bytes(s);
        good = h.offset[s] >= (int64_t)sizeof(Header) && h.bytes[s] == need && h.offset[s] + need <= p->file_bytes;
    }
    if (!good) {
        ::close(fd);
        delete p;
        return fail(GD_ERR_ARG, std::string("gd_pack_open: inconsistent header or truncated file: ") + path);
    }
    if (n) *n = h.n;
    if (dims) {
        dims[0] = h.H;
        dims[1] = h.W;
        dims[2] = h.h;
        dims[3] = h.w;
        dims[4] = h.has_gt;
    }
    *handle = p;
    return GD_OK;
}

long long gd_pack_section_bytes(void* handle, int section) {
    using namespace gd::ingest;
    Pack* p = static_cast<Pack*>(handle);
    if (!p || section < 0 || section >= kSections) return -1;
    return p->hd.bytes[section];
}

int gd_pack_read(void* handle, int section, long long g0, long long count, void* dst, int nthreads) {
    using namespace gd::ingest;
    Pack* p = static_cast<Pack*>(handle);
    if (!p || (!dst && (count > 0 || section == 4))) return fail(GD_ERR_ARG, "gd_pack_read: null argument");
    if (section < 0 || section >= kSections) return fail(GD_ERR_ARG, "gd_pack_read: bad section");
    if (section == 2 && !p->hd.has_gt) return fail(GD_ERR_ARG, "gd_pack_read: file has no ground truth");
    if (section == 4) {  // info JSON, whole
        return pread_all(p->fd, static_cast<char*>(dst), p->hd.offset[4], p->hd.bytes[4])
                   ? GD_OK : fail(GD_ERR_ARG, "gd_pack_read: I/O error");
    }
    if (g0 < 0 || count < 0 || g0 + count > p->hd.n) return fail(GD_ERR_ARG, "gd_pack_read: range out of bounds");
    if (count == 0) return GD_OK;
    const int64_t ib = p->item_bytes(section), off = p->hd.offset[section] + g0 * ib, len = count * ib;
    constexpr int64_t kBlock = int64_t(4) << 20;  // 4 MiB per thread work item
    const int64_t blocks = (len + kBlock - 1) / kBlock;
    char* d = static_cast<char*>(dst);
    const bool ok = parallel_for(blocks, nthreads, [&](int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) {
            const int64_t o = i * kBlock, l = (o + kBlock < len ? kBlock : len - o);
            if (!pread_all(p->fd, d + o, off + o, l)) return false;
        }
        return true;
    });
    return ok ? GD_OK : fail(GD_ERR_ARG, "gd_pack_read: I/O error");
}

int gd_pack_gather(void* handle, int section, const long long* idx, long long count, void* dst, int nthreads) {
    using namespace gd::ingest;
    Pack* p = static_cast<Pack*>(handle);
    if (!p || (!idx && count) || (!dst && count)) return fail(GD_ERR_ARG, "gd_pack_gather: null argument");
    if (section < 0 || section > 3) return fail(GD_ERR_ARG, "gd_pack_gather: bad section");
    if (section == 2 && !p->hd.has_gt) return fail(GD_ERR_ARG, "gd_pack_gather: file has no ground truth");
    for (long long i = 0; i < count; ++i)
        if (idx[i] < 0 || idx[i] >= p->hd.n) return fail(GD_ERR_ARG, "gd_pack_gather: index out of bounds");
    const int64_t ib = p->item_bytes(section);
    char* d = static_cast<char*>(dst);
    const bool ok = parallel_for(count, nthreads, [&](int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i)
            if (!pread_all(p->fd, d + i * ib, p->hd.offset[section] + idx[i] * ib, ib)) return false;
        return true;
    });
    return ok ? GD_OK : fail(GD_ERR_ARG, "gd_pack_gather: I/O error");
}

int gd_pack_close(void* handle) {
    using namespace gd::ingest;
    Pack* p = static_cast<Pack*>(handle);
    if (!p) return GD_OK;
    ::close(p->fd);
    delete p;
    return GD_OK;
}

}  // extern "C"
