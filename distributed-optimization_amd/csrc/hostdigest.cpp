// hostdigest.cpp -- content digest of host arrays on several threads (host code).
//
// The drop-in trainers keep one engine per device with a data set loaded, and reuse it when the
// next trainer's shards have the same CONTENT (trainer._fingerprint: CPython reuses the ids of
// freed arrays, and shards edited in place keep theirs).  At C3 that is 8.6 GB of host shards per
// run; one Python hashing thread reads them at ~6 GB/s, so the digest is computed here instead:
// the arrays are cut into 4 MiB chunks, every chunk is hashed on its own thread (four independent
// multiply-rotate lanes over 32-byte strides, the xxh64 round), and the chunk digests are folded
// in array / chunk order into two 64-bit lanes (a 128-bit digest).  Any change of a byte, of a
// length or of the order of the arrays changes the digest, up to 64-bit collisions per chunk.
#include <stdint.h>
#include <string.h>

#include <sched.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "dopt.h"

namespace {

constexpr uint64_t kP1 = 0x9E3779B185EBCA87ull, kP2 = 0xC2B2AE3D27D4EB4Full, kP3 = 0x165667B19E3779F9ull,
                   kP4 = 0x85EBCA77C2B2AE63ull, kP5 = 0x27D4EB2F165667C5ull;
constexpr int64_t kChunk = 4 << 20;

inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t round1(uint64_t acc, uint64_t w) { return rotl(acc + w * kP2, 31) * kP1; }
inline uint64_t merge(uint64_t h, uint64_t acc) { return (h ^ round1(0, acc)) * kP1 + kP4; }
inline uint64_t avalanche(uint64_t h) {
  h ^= h >> 33;
  h *= kP2;
  h ^= h >> 29;
  h *= kP3;
  return h ^ (h >> 32);
}

// 64-bit digest of n bytes (the xxh64 structure: four lanes, then the tail word by word)
uint64_t chunk_digest(const uint8_t* p, int64_t n, uint64_t seed) {
  int64_t i = 0;
  uint64_t h;
  if (n >= 32) {
    uint64_t a0 = seed + kP1 + kP2, a1 = seed + kP2, a2 = seed, a3 = seed - kP1;
    for (; i + 32 <= n; i += 32) {
      uint64_t w[4];
      memcpy(w, p + i, 32);
      a0 = round1(a0, w[0]);
      a1 = round1(a1, w[1]);
      a2 = round1(a2, w[2]);
      a3 = round1(a3, w[3]);
    }
    h = rotl(a0, 1) + rotl(a1, 7) + rotl(a2, 12) + rotl(a3, 18);
    h = merge(merge(merge(merge(h, a0), a1), a2), a3);
  } else {
    h = seed + kP5;
  }
  h += (uint64_t)n;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    h = rotl(h ^ round1(0, w), 27) * kP1 + kP4;
  }
  for (; i < n; ++i) h = rotl(h ^ (p[i] * kP5), 11) * kP1;
  return avalanche(h);
}

int default_threads() {
  cpu_set_t s;
  int cpus = (int)std::thread::hardware_concurrency();
  if (sched_getaffinity(0, sizeof(s), &s) == 0) cpus = CPU_COUNT(&s);
  int local = 1;  // torchrun: the node's CPUs split over its ranks
  if (const char* v = getenv("LOCAL_WORLD_SIZE")) local = std::max(1, atoi(v));
  return std::max(1, std::min(16, cpus / local));
}

struct Piece {
  int32_t array;
  int64_t off, len;
};

}  // namespace

extern "C" int dopt_host_digest(int32_t n_arrays, const void* const* ptrs, const int64_t* bytes, int32_t threads,
                                uint64_t out[2]) {
  if (n_arrays < 0 || (n_arrays > 0 && (!ptrs || !bytes)) || !out) return DOPT_ERR_INVALID;
  std::vector<Piece> pieces;
  for (int32_t a = 0; a < n_arrays; ++a) {
    if (bytes[a] < 0 || (bytes[a] > 0 && !ptrs[a])) return DOPT_ERR_INVALID;
    for (int64_t o = 0; o < bytes[a]; o += kChunk) pieces.push_back({a, o, std::min<int64_t>(kChunk, bytes[a] - o)});
  }
  std::vector<uint64_t> dig(pieces.size());
  auto run = [&](std::atomic<size_t>* next) {
    for (size_t k; (k = next->fetch_add(1)) < pieces.size();) {
      const Piece& q = pieces[k];
      dig[k] = chunk_digest((const uint8_t*)ptrs[q.array] + q.off, q.len, (uint64_t)q.off);
    }
  };
  std::atomic<size_t> next{0};
  const int nt = (int)std::min<size_t>(pieces.size(), (size_t)(threads > 0 ? threads : default_threads()));
  if (nt <= 1) {
    run(&next);
  } else {
    std::vector<std::thread> th;
    try {
      for (int t = 1; t < nt; ++t) th.emplace_back(run, &next);
    } catch (...) {  // fewer threads than asked: the ones started (and this one) do the rest
    }
    run(&next);
    for (auto& t : th) t.join();
  }
  // fold in order: arrays (index and byte count), then their chunks
  uint64_t h0 = kP5 ^ (uint64_t)n_arrays, h1 = kP3 + (uint64_t)n_arrays;
  size_t k = 0;
  for (int32_t a = 0; a < n_arrays; ++a) {
    h0 = merge(h0, (uint64_t)bytes[a] ^ ((uint64_t)a << 48));
    h1 = merge(h1 ^ 0x5bd1e995u, (uint64_t)bytes[a] + (uint64_t)a);
    for (; k < pieces.size() && pieces[k].array == a; ++k) {
      h0 = merge(h0, dig[k]);
      h1 = merge(rotl(h1, 17), dig[k] ^ kP2);
    }
  }
  out[0] = avalanche(h0);
  out[1] = avalanche(h1 ^ out[0]);
  return DOPT_OK;
}
