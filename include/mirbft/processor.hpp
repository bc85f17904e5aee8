// mirbft/processor.hpp -- C++ host mirror of MirBFT's hash plugin surface,
// backed by libmirsha (include/mirsha.h). Header-only; link with -lmirsha.
//
// Reference (Go), /root/reference/pkg/processor/serial.go:
//
//   type Hasher interface { New() hash.Hash }                                  // :21-23
//   func ProcessHashActions(hasher Hasher, actions *statemachine.ActionList)
//           (*statemachine.EventList, error)                                   // :180-198
//
// plus statemachine.ActionHash / EventHashResult (actions.go:173-187,
// events.go:96-110) and the state.proto hash messages (:78-109, :168-171).
//
// Same names, argument meaning and error behaviour: ProcessHashActions yields
// one HashResult per action in list order, each carrying the SAME origin
// object (shared_ptr identity, the Go pointer), and fails with
// "unexpected type for Hash action: <type>" on a non-hash action
// (serial.go:192-194). The difference is the engine: the whole list is hashed
// by one msha_hash_actions() call (one H2D, one launch per GPU, one D2H).
#pragma once

#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <variant>
#include <vector>

#include "../mirsha.h"

namespace mirbft {

using Bytes = std::vector<uint8_t>;

// ---- state.HashOrigin (protos/state/state.proto:78-104) --------------------
struct RequestAck {
  uint64_t client_id = 0, req_no = 0;
  Bytes digest;
};
struct HashOriginBatch {
  uint64_t source = 0, epoch = 0, seq_no = 0;
  std::vector<RequestAck> request_acks;
};
struct HashOriginVerifyBatch {
  uint64_t source = 0, seq_no = 0;
  std::vector<RequestAck> request_acks;
  Bytes expected_digest;
};
struct HashOriginEpochChange {
  uint64_t source = 0, origin = 0;  // epoch_change payload omitted: only its hash data matters here
};
struct HashOrigin {
  std::variant<std::monostate, HashOriginBatch, HashOriginEpochChange, HashOriginVerifyBatch> type;
};

// ---- state.Action / state.Event (hash members only) ------------------------
struct ActionHashRequest {  // state.proto:168-171
  std::vector<Bytes> data;
  std::shared_ptr<HashOrigin> origin;
};
struct ActionOther {  // any non-hash action (send, persist, commit, ...)
  std::string type_name;
};
struct Action {
  std::variant<ActionHashRequest, ActionOther> type;
};
struct EventHashResult {  // state.proto:106-109
  Bytes digest;
  std::shared_ptr<HashOrigin> origin;
};

namespace statemachine {

class ActionList {
 public:
  ActionList& PushBack(Action a) {
    list_.push_back(std::move(a));
    return *this;
  }
  // ActionList.Hash (actions.go:173-176)
  ActionList& Hash(std::vector<Bytes> data, std::shared_ptr<HashOrigin> origin) {
    return PushBack(Action{ActionHashRequest{std::move(data), std::move(origin)}});
  }
  size_t Len() const { return list_.size(); }
  const std::vector<Action>& Items() const { return list_; }

 private:
  std::vector<Action> list_;
};

class EventList {
 public:
  // EventList.HashResult (events.go:96-99)
  EventList& HashResult(Bytes digest, std::shared_ptr<HashOrigin> origin) {
    list_.push_back(EventHashResult{std::move(digest), std::move(origin)});
    return *this;
  }
  size_t Len() const { return list_.size(); }
  const std::vector<EventHashResult>& Items() const { return list_; }

 private:
  std::vector<EventHashResult> list_;
};

}  // namespace statemachine

namespace processor {

// A Go-style (value, error) result: err empty on success.
template <class T>
struct Result {
  T value;
  std::string err;
  bool ok() const { return err.empty(); }
};

class GPUHasher;

// hash.Hash over the GPU engine: Write appends; Sum(b) appends the digest of
// everything written so far and does not reset (Go hash.Hash semantics).
class GPUHash {
 public:
  explicit GPUHash(GPUHasher* h) : hasher_(h) {}
  size_t Write(const uint8_t* p, size_t n) {
    buf_.insert(buf_.end(), p, p + n);
    return n;
  }
  size_t Write(const Bytes& b) { return Write(b.data(), b.size()); }
  Bytes Sum(Bytes b = {}) const;
  void Reset() { buf_.clear(); }
  static constexpr int Size() { return 32; }
  static constexpr int BlockSize() { return 64; }

 private:
  GPUHasher* hasher_;
  Bytes buf_;
};

// processor.Hasher backed by a libmirsha context (one or more GPUs).
class GPUHasher {
 public:
  explicit GPUHasher(uint32_t device_mask = 1) {
    if (int rc = msha_ctx_create(device_mask, &ctx_); rc != MSHA_OK)
      throw std::runtime_error(std::string("libmirsha: ") + msha_last_error(nullptr));
  }
  ~GPUHasher() { msha_ctx_destroy(ctx_); }
  GPUHasher(const GPUHasher&) = delete;
  GPUHasher& operator=(const GPUHasher&) = delete;

  GPUHash New() { return GPUHash(this); }

  // One digest per message = SHA-256(concat(parts)), in order.
  Result<std::vector<Bytes>> HashBatch(const std::vector<const std::vector<Bytes>*>& msgs) {
    Result<std::vector<Bytes>> r;
    size_t n_parts = 0, n_bytes = 0;
    for (auto* m : msgs) {
      n_parts += m->size();
      for (auto& p : *m) n_bytes += p.size();
    }
    // Pack [][]byte into one arena + offsets: the layout the C ABI takes.
    Bytes arena(n_bytes + 1);
    std::vector<uint64_t> off(n_parts + 1), len(n_parts + 1), begin(msgs.size() + 1);
    size_t pos = 0, j = 0;
    for (size_t i = 0; i < msgs.size(); ++i) {
      begin[i] = j;
      for (auto& p : *msgs[i]) {
        if (!p.empty()) std::memcpy(arena.data() + pos, p.data(), p.size());
        off[j] = pos;
        len[j] = p.size();
        pos += p.size();
        ++j;
      }
    }
    begin[msgs.size()] = j;
    Bytes out(32 * msgs.size());
    if (!msgs.empty()) {
      int rc = msha_hash_actions(ctx_, arena.data(), n_bytes, off.data(), len.data(), n_parts,
                                 begin.data(), msgs.size(), out.data());
      if (rc != MSHA_OK) {
        r.err = "libmirsha error " + std::to_string(rc) + ": " + msha_last_error(ctx_);
        return r;
      }
    }
    r.value.reserve(msgs.size());
    for (size_t i = 0; i < msgs.size(); ++i)  // fresh copies: the state machine keeps digests
      r.value.emplace_back(out.begin() + 32 * i, out.begin() + 32 * (i + 1));
    return r;
  }

  // Batched request intake: Client.Propose's per-call digest
  // (clients.go:189-192) for a whole batch of proposals, one msha_digest_batch.
  Result<std::vector<Bytes>> RequestDigests(const std::vector<Bytes>& requests) {
    Result<std::vector<Bytes>> r;
    size_t total = 0;
    for (auto& q : requests) total += q.size();
    Bytes arena(total + 1);
    std::vector<uint64_t> off(requests.size() + 1), len(requests.size() + 1);
    size_t pos = 0;
    for (size_t i = 0; i < requests.size(); ++i) {
      if (!requests[i].empty()) std::memcpy(arena.data() + pos, requests[i].data(), requests[i].size());
      off[i] = pos;
      len[i] = requests[i].size();
      pos += requests[i].size();
    }
    Bytes out(32 * requests.size());
    if (!requests.empty()) {
      int rc = msha_digest_batch(ctx_, arena.data(), total, off.data(), len.data(), requests.size(),
                                 out.data());
      if (rc != MSHA_OK) {
        r.err = "libmirsha error " + std::to_string(rc) + ": " + msha_last_error(ctx_);
        return r;
      }
    }
    for (size_t i = 0; i < requests.size(); ++i)
      r.value.emplace_back(out.begin() + 32 * i, out.begin() + 32 * (i + 1));
    return r;
  }

  msha_ctx* ctx() { return ctx_; }

 private:
  msha_ctx* ctx_ = nullptr;
};

inline Bytes GPUHash::Sum(Bytes b) const {
  std::vector<Bytes> one{buf_};
  auto r = hasher_->HashBatch({&one});
  if (!r.ok()) throw std::runtime_error(r.err);
  b.insert(b.end(), r.value[0].begin(), r.value[0].end());
  return b;
}

// processor.ProcessHashActions (serial.go:180-198), one GPU batch per list.
inline Result<statemachine::EventList> ProcessHashActions(GPUHasher& hasher,
                                                          const statemachine::ActionList& actions) {
  Result<statemachine::EventList> r;
  std::vector<const ActionHashRequest*> reqs;
  reqs.reserve(actions.Len());
  for (const Action& a : actions.Items()) {
    if (auto* h = std::get_if<ActionHashRequest>(&a.type)) {
      reqs.push_back(h);
    } else {
      r.err = "unexpected type for Hash action: " + std::get<ActionOther>(a.type).type_name;
      return r;
    }
  }
  std::vector<const std::vector<Bytes>*> msgs;
  msgs.reserve(reqs.size());
  for (auto* q : reqs) msgs.push_back(&q->data);
  auto digests = hasher.HashBatch(msgs);
  if (!digests.ok()) {
    r.err = digests.err;
    return r;
  }
  for (size_t i = 0; i < reqs.size(); ++i) r.value.HashResult(std::move(digests.value[i]), reqs[i]->origin);
  return r;
}

}  // namespace processor
}  // namespace mirbft
