// vs_io.hip -- persistence half of the path: faiss flat-file payloads streamed
// straight between the file and HBM.
//
// The reference persists with faiss.write_index / faiss.read_index (utils/vector_store.py:234, :249)
// and rewrites the WHOLE index after every indexer batch (core/indexer.py:945, :970).  Here:
//   * vs_add_from_file reads an IxFI/IxF2 payload (row-major fp32, byte offset given by the host
//     layer's header parser) with parallel pread into two pinned chunks, overlapped with the H2D
//     copy and k_pack_rows of the previous chunk (vs::add_rows_host);
//   * vs_write_rows_to_file writes stored rows back with pwrite, overlapped with the unpack + D2H
//     copy of the next chunk (vs::read_rows_host).  The host layer uses it both for full rewrites
//     and for APPENDS: rows are immutable once added, so a save after new add_item calls only
//     writes the new rows and then the 45-byte header (byte-identical to a full faiss rewrite).
#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/vs.h"
#include "vs_internal.h"

using namespace vs;

namespace {

struct Fd {
    int fd = -1;
    ~Fd() {
        if (fd >= 0) ::close(fd);
    }
};

std::string sys_err(const char* what, const char* path) {
    return std::string(what) + " " + path + ": " + std::strerror(errno);
}

// read exactly `len` bytes at `off` (short reads retried; EOF is an error)
void pread_full(int fd, void* dst, size_t len, int64_t off, const char* path) {
    uint8_t* p = (uint8_t*)dst;
    while (len > 0) {
        const ssize_t r = ::pread(fd, p, len, (off_t)off);
        if (r < 0) {
            if (errno == EINTR) continue;
            throw VsError(VS_ERR_ARG, sys_err("read", path));
        }
        if (r == 0) throw VsError(VS_ERR_ARG, std::string("unexpected end of file in ") + path);
        p += r;
        len -= (size_t)r;
        off += r;
    }
}

void pwrite_full(int fd, const void* src, size_t len, int64_t off, const char* path) {
    const uint8_t* p = (const uint8_t*)src;
    while (len > 0) {
        const ssize_t r = ::pwrite(fd, p, len, (off_t)off);
        if (r < 0) {
            if (errno == EINTR) continue;
            throw VsError(VS_ERR_ARG, sys_err("write", path));
        }
        p += r;
        len -= (size_t)r;
        off += r;
    }
}

// one chunk read by up to kReaders threads (page-cache copies are memcpy-bound per thread)
constexpr int kReaders = 4;
void pread_parallel(int fd, void* dst, size_t len, int64_t off, const char* path) {
    const size_t min_part = 4u << 20;
    const int nt = (int)std::min<size_t>(kReaders, std::max<size_t>(1, len / min_part));
    if (nt <= 1) {
        pread_full(fd, dst, len, off, path);
        return;
    }
    const size_t part = (len / nt + 4095) & ~(size_t)4095;
    std::vector<std::thread> th;
    std::vector<std::string> errs((size_t)nt);
    for (int t = 0; t < nt; ++t) {
        const size_t b = std::min(len, part * t), e = std::min(len, part * (t + 1));
        if (b >= e) break;
        th.emplace_back([&, t, b, e] {
            try {
                pread_full(fd, (uint8_t*)dst + b, e - b, off + (int64_t)b, path);
            } catch (const std::exception& ex) {
                errs[(size_t)t] = ex.what();
            }
        });
    }
    for (auto& x : th) x.join();
    for (auto& m : errs)
        if (!m.empty()) throw VsError(VS_ERR_ARG, m);
}

}  // namespace

extern "C" {

int vs_add_from_file(vs_index* ix, const char* path, int64_t byte_offset, int64_t n) {
    return guarded([&] {
        if (!ix) throw VsError(VS_ERR_ARG, "null index");
        if (!path) throw VsError(VS_ERR_ARG, "path is null");
        if (n < 0 || byte_offset < 0) throw VsError(VS_ERR_ARG, "bad file range");
        if (n == 0) return;
        const int64_t d = vs_dim(ix);
        const int64_t row_bytes = d * (int64_t)sizeof(float);
        Fd f;
        f.fd = ::open(path, O_RDONLY | O_CLOEXEC);
        if (f.fd < 0) throw VsError(VS_ERR_ARG, sys_err("open", path));
        struct stat st;
        if (::fstat(f.fd, &st) != 0) throw VsError(VS_ERR_ARG, sys_err("stat", path));
        if (byte_offset + n * row_bytes > (int64_t)st.st_size)
            throw VsError(VS_ERR_ARG, std::string("file too short for the requested rows: ") + path);
        (void)::posix_fadvise(f.fd, (off_t)byte_offset, (off_t)(n * row_bytes), POSIX_FADV_SEQUENTIAL);
        add_rows_host(ix, n, [&](int64_t r0, int64_t m, float* dst) {
            pread_parallel(f.fd, dst, (size_t)(m * row_bytes), byte_offset + r0 * row_bytes, path);
        });
    });
}

int vs_write_rows_to_file(vs_index* ix, const char* path, int64_t byte_offset, int64_t i0, int64_t n) {
    return guarded([&] {
        if (!ix) throw VsError(VS_ERR_ARG, "null index");
        if (!path) throw VsError(VS_ERR_ARG, "path is null");
        if (n < 0 || i0 < 0 || byte_offset < 0) throw VsError(VS_ERR_ARG, "bad file range");
        if (n == 0) return;
        const int64_t row_bytes = (int64_t)vs_dim(ix) * (int64_t)sizeof(float);
        Fd f;
        f.fd = ::open(path, O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
        if (f.fd < 0) throw VsError(VS_ERR_ARG, sys_err("open", path));
        read_rows_host(ix, i0, n, [&](int64_t r0, int64_t m, const float* src) {
            pwrite_full(f.fd, src, (size_t)(m * row_bytes), byte_offset + r0 * row_bytes, path);
        });
    });
}

}  // extern "C"
