// Memory regions for host-side runtime tables: process-private (anonymous, reserve-only) or
// node-shared (a /dev/shm file every rank of a one-process-per-GPU group maps). Pages are
// committed on first touch in both cases, so a table sized for 16 M accounts costs only what
// is used.
#pragma once
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace igp {

class Region {
 public:
  Region() = default;
  Region(const Region&) = delete;
  Region& operator=(const Region&) = delete;
  Region(Region&& o) noexcept { *this = std::move(o); }
  Region& operator=(Region&& o) noexcept {
    release();
    base_ = o.base_; bytes_ = o.bytes_; path_ = std::move(o.path_); unlink_ = o.unlink_;
    o.base_ = nullptr; o.bytes_ = 0; o.unlink_ = false;
    return *this;
  }
  ~Region() { release(); }

  // anonymous private mapping (MAP_NORESERVE: address space only until touched)
  static Region anon(size_t bytes) {
    Region r;
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (p == MAP_FAILED) throw std::runtime_error("Region: anonymous mmap of " + std::to_string(bytes) + " bytes failed");
    hugepages(p, bytes);
    r.base_ = p;
    r.bytes_ = bytes;
    return r;
  }
  // /dev/shm/<name>: create (sized, zero-filled sparse file) or open an existing one
  static Region shared(const std::string& name, size_t bytes, bool create) {
    if (name.empty() || name.find('/') != std::string::npos) throw std::runtime_error("Region: bad shm name");
    Region r;
    r.path_ = "/dev/shm/" + name;
    const int fd = ::open(r.path_.c_str(), create ? (O_RDWR | O_CREAT | O_EXCL) : O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("Region: open " + r.path_ + ": " + std::strerror(errno));
    if (create) {
      if (::ftruncate(fd, (off_t)bytes) != 0) {
        const int e = errno;
        ::close(fd);
        ::unlink(r.path_.c_str());
        throw std::runtime_error("Region: ftruncate " + r.path_ + ": " + std::strerror(e));
      }
      r.unlink_ = true;
    } else {
      struct stat st;
      if (::fstat(fd, &st) != 0) {
        ::close(fd);
        throw std::runtime_error("Region: fstat " + r.path_);
      }
      if (bytes == 0) bytes = (size_t)st.st_size;
      if ((size_t)st.st_size < bytes) {
        ::close(fd);
        throw std::runtime_error("Region: " + r.path_ + " is smaller than expected");
      }
    }
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_NORESERVE, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("Region: mmap " + r.path_ + " failed");
    hugepages(p, bytes);
    r.base_ = p;
    r.bytes_ = bytes;
    return r;
  }
  // the file name goes away now (mappings stay valid); the creator calls this once every
  // rank has mapped the region
  void unlink() {
    if (!path_.empty()) ::unlink(path_.c_str());
    unlink_ = false;
  }
  // transparent huge pages for large tables: the hash tables are probed at random (an
  // AccountIndex lookup per request row), so with 4 KiB pages nearly every probe also misses the
  // TLB; a no-op where THP is off (shmem THP follows /sys/kernel/mm/transparent_hugepage/shmem_enabled)
  static void hugepages(void* p, size_t bytes) {
    if (bytes >= (size_t(8) << 20)) (void)madvise(p, bytes, MADV_HUGEPAGE);
  }
  void* base() const { return base_; }
  size_t bytes() const { return bytes_; }
  bool shared_mapping() const { return !path_.empty(); }

 private:
  void release() {
    if (base_) munmap(base_, bytes_);
    if (unlink_ && !path_.empty()) ::unlink(path_.c_str());
    base_ = nullptr;
    unlink_ = false;
  }
  void* base_ = nullptr;
  size_t bytes_ = 0;
  std::string path_;
  bool unlink_ = false;
};

}  // namespace igp
