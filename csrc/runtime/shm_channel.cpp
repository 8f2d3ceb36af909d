// Shared-memory control channel of the TP brain (see shm_channel.h).
#include "shm_channel.h"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace vwa {

namespace {
constexpr uint64_t kMagic = 0x7677615f73686d31ull;  // "vwa_shm1"
constexpr int64_t kLine = 64;
// header lines
constexpr int64_t kHMagic = 0, kHReaders = 1, kHSlots = 2, kHSlotBytes = 3, kHSeq = 4, kHBeat = 5, kHdrLines = 8;

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// spin -> yield -> short sleeps: the lockstep peers usually arrive within microseconds of each
// other (spinning gives the ~us hand-off), an idle group must not burn a core
struct Backoff {
  int n = 0;
  void pause() {
    ++n;
    if (n < 2000) {
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    } else if (n < 4000) {
      sched_yield();
    } else {
      const long us = n < 6000 ? 20 : 200;
      std::this_thread::sleep_for(std::chrono::microseconds(us));
    }
  }
};

std::string shm_path(const std::string& name) { return "/dev/shm/" + name; }
}  // namespace

ShmChannel::ShmChannel(const std::string& name, int n_readers, int64_t slot_bytes, int n_slots, bool create)
    : name_(name), n_readers_(n_readers), n_slots_(n_slots), slot_bytes_(slot_bytes), owner_(create) {
  if (name.empty() || name.find('/') != std::string::npos) throw std::invalid_argument("shm channel: bad name");
  if (create && (n_readers < 1 || n_readers > 64 || n_slots < 1 || slot_bytes < 64))
    throw std::invalid_argument("shm channel: 1..64 readers, >= 1 slot of >= 64 bytes");
  const std::string path = shm_path(name);
  int fd = create ? ::open(path.c_str(), O_RDWR | O_CREAT | O_EXCL, 0600) : ::open(path.c_str(), O_RDWR);
  if (fd < 0) throw std::runtime_error("shm channel: cannot open " + path);
  if (create) {
    slot_bytes_ = (slot_bytes + kLine - 1) / kLine * kLine;
    bytes_ = (kHdrLines + n_readers) * kLine + (int64_t)n_slots * (kLine + slot_bytes_);
    if (::ftruncate(fd, bytes_) != 0) {
      ::close(fd);
      ::unlink(path.c_str());
      throw std::runtime_error("shm channel: ftruncate failed");
    }
  } else {
    struct stat st;
    if (::fstat(fd, &st) != 0 || st.st_size < (kHdrLines + 1) * kLine) {
      ::close(fd);
      throw std::runtime_error("shm channel: not initialised");
    }
    bytes_ = st.st_size;
  }
  void* p = ::mmap(nullptr, (size_t)bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("shm channel: mmap failed");
  base_ = static_cast<char*>(p);
  if (create) {
    std::memset(base_, 0, (size_t)bytes_);
    word(kHReaders)->store((uint64_t)n_readers, std::memory_order_relaxed);
    word(kHSlots)->store((uint64_t)n_slots, std::memory_order_relaxed);
    word(kHSlotBytes)->store((uint64_t)slot_bytes_, std::memory_order_relaxed);
    word(kHBeat)->store(now_ns(), std::memory_order_relaxed);
    word(kHMagic)->store(kMagic, std::memory_order_release);  // last: readers check it
  } else {
    // (a reader may attach before the leader finished initialising: wait for the magic, bounded)
    Backoff b;
    const uint64_t t0 = now_ns();
    while (word(kHMagic)->load(std::memory_order_acquire) != kMagic) {
      if (now_ns() - t0 > 10ull * 1000000000ull) {
        ::munmap(base_, (size_t)bytes_);
        throw std::runtime_error("shm channel: leader never initialised " + path);
      }
      b.pause();
    }
    n_readers_ = (int)word(kHReaders)->load(std::memory_order_relaxed);
    n_slots_ = (int)word(kHSlots)->load(std::memory_order_relaxed);
    slot_bytes_ = (int64_t)word(kHSlotBytes)->load(std::memory_order_relaxed);
    if ((kHdrLines + n_readers_) * kLine + (int64_t)n_slots_ * (kLine + slot_bytes_) > bytes_)
      throw std::runtime_error("shm channel: size mismatch");
  }
}

ShmChannel::~ShmChannel() {
  if (base_) ::munmap(base_, (size_t)bytes_);
  if (owner_ && !unlinked_) ::unlink(shm_path(name_).c_str());
}

std::atomic<uint64_t>* ShmChannel::word(int64_t line) const {
  return reinterpret_cast<std::atomic<uint64_t>*>(base_ + line * kLine);
}

char* ShmChannel::slot(int64_t k) const {
  const int64_t i = (k - 1) % n_slots_;
  return base_ + (kHdrLines + n_readers_) * kLine + i * (kLine + slot_bytes_);
}

void ShmChannel::beat() { word(kHBeat)->store(now_ns(), std::memory_order_release); }

void ShmChannel::unlink() {
  if (owner_ && !unlinked_) {
    ::unlink(shm_path(name_).c_str());
    unlinked_ = true;
  }
}

int64_t ShmChannel::published() const { return (int64_t)word(kHSeq)->load(std::memory_order_acquire); }

int64_t ShmChannel::acked(int r) const {
  if (r < 0 || r >= n_readers_) throw std::out_of_range("shm channel: reader index");
  return (int64_t)word(kHdrLines + r)->load(std::memory_order_acquire);
}

int64_t ShmChannel::publish(const std::string& payload, double timeout_s) {
  if ((int64_t)payload.size() > slot_bytes_) throw std::length_error("shm channel: message exceeds the slot size");
  const int64_t k = (int64_t)word(kHSeq)->load(std::memory_order_relaxed) + 1;
  // the slot is free once every reader consumed message k - n_slots
  Backoff b;
  const uint64_t t0 = now_ns();
  for (int r = 0; r < n_readers_; ++r) {
    while ((int64_t)word(kHdrLines + r)->load(std::memory_order_acquire) < k - n_slots_) {
      if (timeout_s >= 0 && (double)(now_ns() - t0) * 1e-9 > timeout_s)
        throw std::runtime_error("shm channel: reader " + std::to_string(r) + " stopped consuming");
      b.pause();
    }
  }
  char* s = slot(k);
  const uint64_t n = payload.size();
  std::memcpy(s + kLine, payload.data(), n);
  reinterpret_cast<std::atomic<uint64_t>*>(s)->store(n, std::memory_order_relaxed);
  word(kHBeat)->store(now_ns(), std::memory_order_relaxed);
  word(kHSeq)->store((uint64_t)k, std::memory_order_release);  // payload + length before seq
  return k;
}

std::string ShmChannel::receive(int r, double timeout_s, double dead_s) {
  if (r < 0 || r >= n_readers_ || r >= 64) throw std::out_of_range("shm channel: reader index");
  int64_t& last = last_[r];
  if (last == 0) last = (int64_t)word(kHdrLines + r)->load(std::memory_order_relaxed);
  const int64_t k = last + 1;
  Backoff b;
  const uint64_t t0 = now_ns();
  while ((int64_t)word(kHSeq)->load(std::memory_order_acquire) < k) {
    const uint64_t t = now_ns();
    if (timeout_s >= 0 && (double)(t - t0) * 1e-9 > timeout_s) throw std::runtime_error("shm channel: receive timed out");
    if (dead_s > 0 && (b.n & 1023) == 0) {
      const uint64_t hb = word(kHBeat)->load(std::memory_order_acquire);
      if (t > hb && (double)(t - hb) * 1e-9 > dead_s)
        throw std::runtime_error("shm channel: leader silent for " + std::to_string(dead_s) + " s (no message, no heartbeat)");
    }
    b.pause();
  }
  const char* s = slot(k);
  const uint64_t n = reinterpret_cast<const std::atomic<uint64_t>*>(s)->load(std::memory_order_relaxed);
  if ((int64_t)n > slot_bytes_) throw std::runtime_error("shm channel: corrupt slot length");
  std::string out(s + kLine, s + kLine + n);
  last = k;
  word(kHdrLines + r)->store((uint64_t)k, std::memory_order_release);
  return out;
}

}  // namespace vwa
