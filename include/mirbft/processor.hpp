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
// by one msha_digest_batch() call over a pinned, 16-byte aligned arena
// (one H2D DMA, one launch per GPU, one D2H).
#pragma once

#include <cstdint>
#include <cstring>
#include <map>
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
  uint64_t source = 0, origin = 0;
  // The *msgs.EpochChange the hash data was built from, by identity only (its
  // fields are not needed here): actions sharing one message share a payload.
  std::shared_ptr<const void> epoch_change;
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
  ~GPUHasher() {
    if (pinned_) msha_pinned_free(ctx_, pinned_);
    msha_ctx_destroy(ctx_);
  }
  GPUHasher(const GPUHasher&) = delete;
  GPUHasher& operator=(const GPUHasher&) = delete;

  GPUHash New() { return GPUHash(this); }

  // One digest per message = SHA-256(concat(parts)), in order. Each message's
  // parts are packed back to back (h.Write appends), every message starting
  // 16-byte aligned, into the context's pinned arena: libmirsha uploads it as
  // is (msha_pinned_alloc / msha_stats.direct_calls), one msha_digest_batch.
  // alias (optional, one entry per message): an earlier message with the same
  // bytes, or -1; such a message is not packed again but shares that one's
  // (off, len), so its payload crosses PCIe once.
  Result<std::vector<Bytes>> HashBatch(const std::vector<const std::vector<Bytes>*>& msgs,
                                       const std::vector<int64_t>* alias = nullptr) {
    Result<std::vector<Bytes>> r;
    size_t n_bytes = 0;
    for (size_t i = 0; i < msgs.size(); ++i) {
      if (alias && (*alias)[i] >= 0) continue;
      for (auto& p : *msgs[i]) n_bytes += p.size();
      n_bytes += 15;
    }
    std::vector<uint64_t> off(msgs.size() + 1), len(msgs.size() + 1);
    uint8_t* arena = nullptr;
    if (!PinnedArena(n_bytes + 64, &arena, &r.err)) return r;
    size_t pos = 0;
    for (size_t i = 0; i < msgs.size(); ++i) {
      if (alias && (*alias)[i] >= 0) {
        off[i] = off[(*alias)[i]];
        len[i] = len[(*alias)[i]];
        continue;
      }
      off[i] = pos;
      for (auto& p : *msgs[i]) {
        if (!p.empty()) std::memcpy(arena + pos, p.data(), p.size());
        pos += p.size();
      }
      len[i] = pos - off[i];
      pos = (pos + 15) & ~size_t(15);
    }
    return Digest(arena, pos, off, len, msgs.size());
  }

  // Batched request intake: Client.Propose's per-call digest
  // (clients.go:189-192) for a whole batch of proposals, one msha_digest_batch.
  Result<std::vector<Bytes>> RequestDigests(const std::vector<Bytes>& requests) {
    std::vector<std::vector<Bytes>> one(requests.size());
    std::vector<const std::vector<Bytes>*> msgs(requests.size());
    for (size_t i = 0; i < requests.size(); ++i) {
      one[i].push_back(requests[i]);
      msgs[i] = &one[i];
    }
    return HashBatch(msgs);
  }

  msha_ctx* ctx() { return ctx_; }

 private:
  // The context's pinned packing arena, grown on demand.
  bool PinnedArena(size_t bytes, uint8_t** p, std::string* err) {
    if (bytes > pinned_cap_) {
      if (pinned_) msha_pinned_free(ctx_, pinned_);
      pinned_ = nullptr;
      pinned_cap_ = 0;
      const size_t want = bytes + bytes / 4 + 4096;
      if (int rc = msha_pinned_alloc(ctx_, want, &pinned_); rc != MSHA_OK) {
        *err = "libmirsha error " + std::to_string(rc) + ": " + msha_last_error(ctx_);
        return false;
      }
      pinned_cap_ = want;
    }
    *p = static_cast<uint8_t*>(pinned_);
    return true;
  }

  Result<std::vector<Bytes>> Digest(const uint8_t* arena, size_t arena_len, const std::vector<uint64_t>& off,
                                    const std::vector<uint64_t>& len, size_t n) {
    Result<std::vector<Bytes>> r;
    Bytes out(32 * n);
    if (n) {
      int rc = msha_digest_batch(ctx_, arena, arena_len, off.data(), len.data(), n, out.data());
      if (rc != MSHA_OK) {
        r.err = "libmirsha error " + std::to_string(rc) + ": " + msha_last_error(ctx_);
        return r;
      }
    }
    r.value.reserve(n);
    for (size_t i = 0; i < n; ++i)  // fresh copies: the state machine keeps digests
      r.value.emplace_back(out.begin() + 32 * i, out.begin() + 32 * (i + 1));
    return r;
  }

  msha_ctx* ctx_ = nullptr;
  void* pinned_ = nullptr;
  size_t pinned_cap_ = 0;
};

inline Bytes GPUHash::Sum(Bytes b) const {
  std::vector<Bytes> one{buf_};
  auto r = hasher_->HashBatch({&one});
  if (!r.ok()) throw std::runtime_error(r.err);
  b.insert(b.end(), r.value[0].begin(), r.value[0].end());
  return b;
}

// The Go drop-in's epochChangeAliases (gpuhash.go): alias[i] = an earlier
// request carrying request i's EpochChange payload, else -1. Each origin's
// EpochChange is hashed once per ack (epoch_target.go:486-528): the same
// message object is the same payload (the testengine passes it by pointer,
// recorder.go:39-47); an equal payload from the same origin node with the same
// length (an ack off the wire) is found by comparing bytes; an altered copy is
// packed and hashed on its own.
inline std::vector<int64_t> EpochChangeAliases(const std::vector<const ActionHashRequest*>& reqs) {
  std::vector<int64_t> alias(reqs.size(), -1);
  std::map<const void*, int64_t> by_obj;
  std::map<std::pair<uint64_t, size_t>, std::vector<int64_t>> by_content;
  auto concat = [](const std::vector<Bytes>& parts) {
    Bytes b;
    for (auto& p : parts) b.insert(b.end(), p.begin(), p.end());
    return b;
  };
  for (size_t i = 0; i < reqs.size(); ++i) {
    const auto* o = reqs[i]->origin ? std::get_if<HashOriginEpochChange>(&reqs[i]->origin->type) : nullptr;
    if (!o) continue;
    const void* key = o->epoch_change.get();
    auto parts_len = [](const std::vector<Bytes>& parts) {
      size_t n = 0;
      for (auto& p : parts) n += p.size();
      return n;
    };
    if (key) {
      // the same message names the same payload only if the Data built from it is
      // the same (the contract is SHA-256(Data), batch_tracker.go:192-195): part for
      // part equal, else the concatenations
      auto it = by_obj.find(key);
      if (it != by_obj.end() && parts_len(reqs[it->second]->data) == parts_len(reqs[i]->data) &&
          (reqs[it->second]->data == reqs[i]->data || concat(reqs[it->second]->data) == concat(reqs[i]->data))) {
        alias[i] = it->second;
        continue;
      }
    }
    const Bytes mine = concat(reqs[i]->data);
    auto& cands = by_content[{o->origin, mine.size()}];
    for (int64_t j : cands)
      if (concat(reqs[j]->data) == mine) {
        alias[i] = j;
        break;
      }
    if (key) by_obj[key] = alias[i] >= 0 ? alias[i] : (int64_t)i;
    if (alias[i] < 0) cands.push_back((int64_t)i);
  }
  return alias;
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
  const std::vector<int64_t> alias = EpochChangeAliases(reqs);
  auto digests = hasher.HashBatch(msgs, &alias);
  if (!digests.ok()) {
    r.err = digests.err;
    return r;
  }
  for (size_t i = 0; i < reqs.size(); ++i) r.value.HashResult(std::move(digests.value[i]), reqs[i]->origin);
  return r;
}

}  // namespace processor
}  // namespace mirbft
