// C++ parity test for the reference-shaped host mirror (include/mirbft/processor.hpp).
// Reads like the reference's ginkgo specs for the processor: Describe
// ProcessHashActions -> It "..." -> Expect. The checker is the CPU oracle
// (oracle/sha256_oracle.c, linked as test infrastructure only).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>

#include "mirbft/processor.hpp"

extern "C" void oracle_sha256(const uint8_t* p, uint64_t n, uint8_t out[32]);

using namespace mirbft;
using mirbft::statemachine::ActionList;

static int failures = 0;
#define EXPECT(cond, what)                                                  \
  do {                                                                      \
    if (!(cond)) {                                                          \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, what);   \
      ++failures;                                                           \
    }                                                                       \
  } while (0)

static Bytes hex(const char* h) {
  Bytes b;
  for (size_t i = 0; h[i] && h[i + 1]; i += 2) b.push_back((uint8_t)std::stoi(std::string(h + i, 2), nullptr, 16));
  return b;
}
static Bytes str(const char* s) { return Bytes(s, s + std::strlen(s)); }
static Bytes oracle(const std::vector<Bytes>& parts) {
  Bytes all;
  for (auto& p : parts) all.insert(all.end(), p.begin(), p.end());
  Bytes d(32);
  oracle_sha256(all.data(), all.size(), d.data());
  return d;
}

int main() {
  processor::GPUHasher hasher(1);

  // Describe("ProcessHashActions")
  {  // It("hashes the FIPS 180-4 examples")
    ActionList al;
    al.Hash({}, nullptr);
    al.Hash({str("abc")}, nullptr);
    al.Hash({str("abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq")}, nullptr);
    auto r = processor::ProcessHashActions(hasher, al);
    EXPECT(r.ok(), "no error");
    EXPECT(r.value.Len() == 3, "one result per action");
    EXPECT(r.value.Items()[0].digest == hex("e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"), "empty");
    EXPECT(r.value.Items()[1].digest == hex("ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"), "abc");
    EXPECT(r.value.Items()[2].digest == hex("248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"), "448-bit");
  }
  {  // It("streams parts like h.Write and keeps order and origin identity")
    std::mt19937_64 rng(42);
    ActionList al;
    std::vector<std::shared_ptr<HashOrigin>> origins;
    std::vector<std::vector<Bytes>> parts_of;
    for (int i = 0; i < 2000; ++i) {
      auto o = std::make_shared<HashOrigin>();
      o->type = HashOriginBatch{0, 1, (uint64_t)i, {}};
      std::vector<Bytes> parts(rng() % 6);
      for (auto& p : parts) {
        p.resize(rng() % 300);
        for (auto& c : p) c = (uint8_t)rng();
      }
      origins.push_back(o);
      parts_of.push_back(parts);
      al.Hash(parts, o);
    }
    auto r = processor::ProcessHashActions(hasher, al);
    EXPECT(r.ok(), "no error");
    EXPECT(r.value.Len() == 2000, "one result per action");
    for (int i = 0; i < 2000 && i < (int)r.value.Len(); ++i) {
      EXPECT(r.value.Items()[i].origin.get() == origins[i].get(), "same origin pointer");
      EXPECT(r.value.Items()[i].digest == oracle(parts_of[i]), "digest == oracle");
    }
  }
  {  // It("fails on a non-hash action with the reference's message")
    ActionList al;
    al.Hash({str("x")}, nullptr);
    al.PushBack(Action{ActionOther{"*state.Action_Send"}});
    auto r = processor::ProcessHashActions(hasher, al);
    EXPECT(!r.ok(), "error returned");
    EXPECT(r.err == "unexpected type for Hash action: *state.Action_Send", "error text");
  }
  {  // It("returns an empty list for an empty list")
    auto r = processor::ProcessHashActions(hasher, ActionList{});
    EXPECT(r.ok() && r.value.Len() == 0, "empty");
  }
  {  // Describe("GPUHash") It("appends on Sum and does not reset")
    auto h = hasher.New();
    h.Write(str("ab"));
    h.Write(str("c"));
    EXPECT(h.Sum() == hex("ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"), "abc");
    Bytes pre = str("pre");
    Bytes s = h.Sum(pre);
    EXPECT(s.size() == 35 && Bytes(s.begin(), s.begin() + 3) == pre, "Sum(b) appends");
  }
  {  // Describe("RequestDigests") It("matches Client.Propose's per-request digest")
    std::vector<Bytes> reqs;
    for (int i = 0; i < 300; ++i) reqs.push_back(Bytes(i * 7 % 600, (uint8_t)i));
    auto r = hasher.RequestDigests(reqs);
    EXPECT(r.ok() && r.value.size() == reqs.size(), "one digest per request");
    for (size_t i = 0; i < reqs.size() && i < r.value.size(); ++i)
      EXPECT(r.value[i] == oracle({reqs[i]}), "request digest == oracle");
  }
  {  // It("packs the list into a pinned, 16-byte aligned arena: a short list takes the
     //     latency path (packed, one H2D), a longer one is uploaded as is")
    msha_stats before{}, after{};
    msha_get_stats(hasher.ctx(), &before);
    ActionList al;
    for (int i = 0; i < 300; ++i) al.Hash({Bytes(i % 97, (uint8_t)i), Bytes(i % 13, 7)}, nullptr);
    auto r = processor::ProcessHashActions(hasher, al);
    EXPECT(r.ok(), "no error");
    msha_get_stats(hasher.ctx(), &after);
    EXPECT(after.small_calls == before.small_calls + 1 && after.direct_calls == before.direct_calls,
           "short list: latency path, packed");
    for (int i = 0; i < 300; ++i)
      EXPECT(r.value.Items()[i].digest == oracle({Bytes(i % 97, (uint8_t)i), Bytes(i % 13, 7)}), "digest");
    ActionList big;  // ~1.3 MB of payload: over the 512 KiB a pinned arena is packed below
    for (int i = 0; i < 3000; ++i) big.Hash({Bytes(400 + i % 50, (uint8_t)i), Bytes(i % 13, 9)}, nullptr);
    before = after;
    auto r2 = processor::ProcessHashActions(hasher, big);
    EXPECT(r2.ok(), "no error");
    msha_get_stats(hasher.ctx(), &after);
    EXPECT(after.direct_calls == before.direct_calls + 1, "longer list: direct (zero-copy) upload");
    for (int i = 0; i < 3000; i += 7)
      EXPECT(r2.value.Items()[i].digest == oracle({Bytes(400 + i % 50, (uint8_t)i), Bytes(i % 13, 9)}), "digest");
  }
  {  // Describe("epoch-change storm") It("packs each distinct EpochChange payload once")
     // Every node hashes each origin's EpochChange once per ack (epoch_target.go:486-528):
     // acks of one message share it (the testengine passes it by pointer), equal copies
     // off the wire share it by content, an altered copy is hashed on its own.
    const int nodes = 12;
    ActionList al;
    std::vector<std::vector<Bytes>> parts_of;
    uint64_t distinct = 0;
    for (int o = 0; o < nodes; ++o) {
      std::vector<Bytes> data{Bytes(8, (uint8_t)o), Bytes(332, (uint8_t)(o + 1))};
      for (int e = 0; e < 2000 + 300 * o; ++e) data.push_back(Bytes(48, (uint8_t)(e ^ o)));
      auto msg = std::make_shared<int>(o);  // the message's identity
      uint64_t bytes = 0;
      for (auto& p : data) bytes += p.size();
      distinct += 2 * ((bytes + 15) / 16 * 16);  // the message and its altered copy
      for (int src = 0; src < nodes; ++src) {
        auto origin = std::make_shared<HashOrigin>();
        HashOriginEpochChange ec{(uint64_t)src, (uint64_t)o, src % 3 == 1 ? std::make_shared<int>(o) : msg};
        origin->type = ec;
        al.Hash(data, origin);
        parts_of.push_back(data);
      }
      std::vector<Bytes> bad = data;
      bad.back()[0] ^= 1;
      auto origin = std::make_shared<HashOrigin>();
      origin->type = HashOriginEpochChange{99, (uint64_t)o, std::make_shared<int>(o)};
      al.Hash(bad, origin);
      parts_of.push_back(bad);
    }
    auto r = processor::ProcessHashActions(hasher, al);
    EXPECT(r.ok(), "no error");
    for (size_t i = 0; i < parts_of.size() && i < r.value.Len(); ++i)
      EXPECT(r.value.Items()[i].digest == oracle(parts_of[i]), "storm digest == oracle");
    uint32_t shards = 0;
    uint64_t up = 0;
    msha_shard_count(hasher.ctx(), &shards);
    for (uint32_t k = 0; k < shards; ++k) {
      msha_shard_stats st{};
      msha_get_shard_stats(hasher.ctx(), k, &st);
      up += st.h2d_payload_bytes;
    }
    EXPECT(up >= distinct - 16 * 2 * nodes && up <= distinct, "each distinct payload uploaded once");
  }
  {  // It("does not alias two actions on one message whose Data differ at equal length")
     // (the contract is SHA-256(Data): batch_tracker.go:192-195)
    auto msg = std::make_shared<int>(7);
    std::vector<Bytes> a{Bytes(8, 1), Bytes(332, 2)}, b{Bytes(8, 3), Bytes(332, 2)}, c{Bytes(8, 1), Bytes(332, 4)};
    ActionList al;
    std::vector<const ActionHashRequest*> reqs;
    for (auto* d : {&a, &b, &c, &a}) {
      auto origin = std::make_shared<HashOrigin>();
      origin->type = HashOriginEpochChange{0, 1, msg};
      al.Hash(*d, origin);
    }
    for (auto& it : al.Items()) reqs.push_back(&std::get<ActionHashRequest>(it.type));
    const auto alias = processor::EpochChangeAliases(reqs);
    EXPECT(alias == std::vector<int64_t>({-1, -1, -1, 0}), "aliases only the equal Data");
    auto r = processor::ProcessHashActions(hasher, al);
    EXPECT(r.ok(), "no error");
    int k = 0;
    for (auto* d : {&a, &b, &c, &a})
      EXPECT(r.ok() && r.value.Items()[k++].digest == oracle(*d), "same pointer, distinct Data: distinct digests");
  }
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("cpp processor mirror: all specs passed\n");
  return 0;
}
