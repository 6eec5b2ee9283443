// sampler.cpp -- legacy-MT19937 minibatch sampler (host code).
//
// Worker.get_mini_batch draws idx = np.random.choice(m, b, replace=False)
// (worker.py:27) from numpy's global RandomState.  In numpy's legacy path that is
// permutation(m)[:b]: a full Fisher-Yates shuffle of arange(m) driven by
// random_interval(i) (masked rejection on 32-bit MT19937 outputs), i = m-1 .. 1.
// This file restates that algorithm so the engine can produce the same index
// stream for T rounds x N workers in one call, reading and writing numpy's
// state words (key[624], pos) in place.  The draw is inherently sequential
// (one global stream, data-dependent rejection counts), so it stays on the host.
#include <stdint.h>
#include <string.h>

#include <sched.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <thread>
#include <vector>

#include "dopt.h"

namespace {

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

// numpy's legacy generator state with a block of tempered outputs: each twist regenerates
// the 624 state words and tempers them in one vectorisable pass, so a draw is a load.
struct MT {
  uint32_t* key;
  int32_t pos;
  uint32_t out[kN];
  int32_t out_gen = -1;  // out[] holds the tempered words of the current key (valid from pos on)

  void twist() {
    int i = 0;
    for (; i < kN - kM; ++i) {
      const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
      key[i] = key[i + kM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    }
    for (; i < kN - 1; ++i) {
      const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
      key[i] = key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    }
    const uint32_t y = (key[kN - 1] & kUpper) | (key[0] & kLower);
    key[kN - 1] = key[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    pos = 0;
  }
  void temper_all() {
    for (int k = 0; k < kN; ++k) {
      uint32_t y = key[k];
      y ^= (y >> 11);
      y ^= (y << 7) & 0x9d2c5680u;
      y ^= (y << 15) & 0xefc60000u;
      y ^= (y >> 18);
      out[k] = y;
    }
    out_gen = 0;
  }
  inline uint32_t next32() {
    if (pos >= kN) {
      twist();
      temper_all();
    } else if (out_gen < 0) {
      temper_all();  // first draw from a state handed in mid-block
    }
    return out[pos++];
  }
  uint64_t next64() {
    const uint64_t hi = next32();
    return (hi << 32) | next32();
  }
  // uniform integer in [0, max] by masked rejection (numpy random_interval)
  inline uint64_t interval(uint64_t max) {
    if (max == 0) return 0;
    uint64_t v;
    if (max <= 0xffffffffull) {
      const uint32_t mask = 0xffffffffu >> __builtin_clz((uint32_t)max);
      while ((v = (next32() & mask)) > max) {
      }
    } else {
      const uint64_t mask = ~0ull >> __builtin_clzll(max);
      while ((v = (next64() & mask)) > max) {
      }
    }
    return v;
  }
};

// The rejection filter (numpy random_interval, masked rejection) over a buffer of tempered
// words, as a branchless scan: a word is kept when (w & mask) <= k, and then k moves on;
// k < 2^32 (m < 2^31 is checked by the callers).  The mask only changes when k drops below a
// power of two, so the scan runs over segments of constant mask, and within a segment 8 words
// at a time without exit tests while k stays >= 8 above the segment's floor (each word lowers
// k by at most 1): the loop-carried chain per word is compare + subtract.  Every candidate is
// recorded in js (the kept ones end up at js[0 .. m-2], js[t] the j of Fisher-Yates step
// k = m-1-t).  This container, interleaved: C3 shape 5.4 -> 4.1 ns per draw with the
// generation inline.
inline void filter_block(const uint32_t* out, int32_t& q, uint32_t& k, uint32_t& t, uint32_t* js) {
  while (q < kN && k >= 1) {
    const uint32_t mask = 0xffffffffu >> __builtin_clz(k);
    const uint32_t klo = mask >> 1;  // the mask holds while k > klo
    while (q + 8 <= kN && k - klo >= 8) {
#pragma GCC unroll 8
      for (int u = 0; u < 8; ++u) {
        const uint32_t v = out[q + u] & mask;
        const uint32_t keep = v <= k;
        js[t] = v;
        t += keep;
        k -= keep;
      }
      q += 8;
    }
    while (q < kN && k > klo) {
      const uint32_t v = out[q++] & mask;
      const uint32_t keep = v <= k;
      js[t] = v;
      t += keep;
      k -= keep;
    }
  }
}

// The j of every Fisher-Yates step k = m-1 .. 1, consuming the stream exactly as m-1 calls of
// interval(k) would.
void draw_js(MT& mt, int64_t m, uint32_t* js) {
  uint32_t k = (uint32_t)(m - 1), t = 0;
  while (k >= 1) {
    if (mt.pos >= kN) {
      mt.twist();
      mt.temper_all();
    } else if (mt.out_gen < 0) {
      mt.temper_all();
    }
    int32_t q = mt.pos;
    filter_block(mt.out, q, k, t, js);
    mt.pos = q;
  }
}

// Fisher-Yates over arange(m) from the recorded js; permutation(m)[:eb] -> out.
template <typename I>
void shuffle_prefix(int64_t m, int64_t eb, const uint32_t* js, std::vector<int64_t>& perm, I* out) {
  perm.resize((size_t)m);
  int64_t* p = perm.data();
  for (int64_t k = 0; k < m; ++k) p[k] = k;
  for (int64_t k = m - 1, t = 0; k >= 1; --k, ++t) {
    const int64_t j = js[(size_t)t];
    const int64_t v = p[k];
    p[k] = p[j];
    p[j] = v;
  }
  for (int64_t k = 0; k < eb; ++k) out[k] = (I)p[k];
}

// permutation(m)[:eb] -> out; perm / js are scratch of size m.
template <typename I>
void choice_prefix(MT& mt, int64_t m, int64_t eb, std::vector<int64_t>& perm, std::vector<uint32_t>& js, I* out) {
  js.resize((size_t)m);
  draw_js(mt, m, js.data());
  shuffle_prefix(m, eb, js.data(), perm, out);
}

// Many draws (T rounds x N workers): the stream's blocks -- twist + temper of 624 words, a
// sequential chain of its own -- are produced by a helper thread into a ring while this thread
// runs the filter, so the caller's critical path is the filter (and the shuffles) alone.  Each
// slot keeps the state words it was tempered from, so the state handed back is exactly the one
// at the consumer's position (blocks made ahead of it are discarded).
class BlockRing {
 public:
  static constexpr int64_t kSlots = 64;
  BlockRing(const uint32_t* key, int32_t pos) : keys_((size_t)kSlots * kN), outs_((size_t)kSlots * kN), pos0_(pos) {
    memcpy(keys_.data(), key, sizeof(uint32_t) * kN);  // slot 0: the current block, not twisted
    temper(keys_.data(), outs_.data());
    produced_.store(1, std::memory_order_release);
    gen_ = std::thread([this] { produce(); });
  }
  ~BlockRing() {
    stop_.store(true, std::memory_order_release);
    gen_.join();
  }
  // tempered words of block b (blocks are consumed in order; b - 1 is released)
  const uint32_t* block(int64_t b) {
    consumed_.store(b, std::memory_order_release);
    while (produced_.load(std::memory_order_acquire) <= b) std::this_thread::yield();
    return outs_.data() + (size_t)(b % kSlots) * kN;
  }
  const uint32_t* key_of(int64_t b) const { return keys_.data() + (size_t)(b % kSlots) * kN; }
  int32_t pos0() const { return pos0_; }

 private:
  static void temper(const uint32_t* key, uint32_t* out) {
    for (int k = 0; k < kN; ++k) {
      uint32_t y = key[k];
      y ^= (y >> 11);
      y ^= (y << 7) & 0x9d2c5680u;
      y ^= (y << 15) & 0xefc60000u;
      y ^= (y >> 18);
      out[k] = y;
    }
  }
  void produce() {
    uint32_t key[kN];
    memcpy(key, keys_.data(), sizeof(key));
    for (int64_t b = 1;; ++b) {
      while (b - consumed_.load(std::memory_order_acquire) >= kSlots) {  // slot b % kSlots still in use
        if (stop_.load(std::memory_order_acquire)) return;
        std::this_thread::yield();
      }
      if (stop_.load(std::memory_order_acquire)) return;
      MT mt{key, 0};
      mt.twist();
      uint32_t* k = keys_.data() + (size_t)(b % kSlots) * kN;
      memcpy(k, key, sizeof(key));
      temper(k, outs_.data() + (size_t)(b % kSlots) * kN);
      produced_.store(b + 1, std::memory_order_release);
    }
  }
  std::vector<uint32_t> keys_, outs_;
  int32_t pos0_;
  std::atomic<int64_t> produced_{0}, consumed_{0};
  std::atomic<bool> stop_{false};
  std::thread gen_;
};

// The consumer side of a BlockRing: the filter over block after block.
struct RingStream {
  BlockRing& ring;
  int64_t b = 0;
  int32_t pos;
  const uint32_t* out;
  explicit RingStream(BlockRing& r) : ring(r), pos(r.pos0()), out(r.block(0)) {}
  void draw(int64_t m, uint32_t* js) {  // m - 1 draws (a permutation of m)
    uint32_t k = (uint32_t)(m - 1), t = 0;
    while (k >= 1) {
      if (pos >= kN) {
        out = ring.block(++b);
        pos = 0;
      }
      filter_block(out, pos, k, t, js);
    }
  }
  void save(uint32_t key[kN], int32_t* p) const {  // numpy's state at this position
    memcpy(key, ring.key_of(b), sizeof(uint32_t) * kN);
    *p = pos;
  }
};

}  // namespace

extern "C" int dopt_mt_choice(uint32_t key[624], int32_t* pos, int64_t m, int64_t b, int64_t* out) {
  if (!key || !pos || m < 0 || m > 0x7fffffffLL || b < 0 || *pos < 0 || *pos > kN) return DOPT_ERR_INVALID;
  if (m == 0) return DOPT_OK;  // worker.py:17-18: no draw for an empty shard
  const int64_t eb = b < m ? b : m;
  if (eb <= 0) return DOPT_OK;  // worker.py:21-23
  MT mt{key, *pos};
  std::vector<int64_t> perm;
  std::vector<uint32_t> js;
  choice_prefix(mt, m, eb, perm, js, out);
  *pos = mt.pos;
  return DOPT_OK;
}

static int check_rounds(const uint32_t* key, const int32_t* pos, int64_t T, int64_t n_workers,
                        const int64_t* shard_rows) {
  if (!key || !pos || T < 0 || n_workers < 0 || *pos < 0 || *pos > kN) return DOPT_ERR_INVALID;
  if (n_workers > 0 && !shard_rows) return DOPT_ERR_INVALID;
  for (int64_t i = 0; i < n_workers; ++i)
    if (shard_rows[i] < 0 || shard_rows[i] > 0x7fffffffLL) return DOPT_ERR_INVALID;
  return DOPT_OK;
}

// Fisher-Yates shuffles of finished filters, off the filter's thread.  Jobs q = (t, i) in draw
// order are grouped in batches of B; batch k's js go to ring slot k % R and are shuffled by
// thread k % H, which publishes how many of its batches are done; the filter overwrites slot
// k % R only once batch k - R is done.  One release/acquire hand-off per batch, not per job.
class ShufflePool {
 public:
  ShufflePool(int64_t T, int64_t n, const int64_t* rows, int64_t b, int32_t* out, int64_t max_m)
      : n_(n), rows_(rows), b_(b), out_(out), stride_(max_m), njobs_(T * n),
        B_(std::max<int64_t>(1, (int64_t(1) << 15) / max_m)), nbatch_((njobs_ + B_ - 1) / B_),
        js_((size_t)(kSlots * B_ * stride_)) {
    try {
      for (int h = 0; h < kThreads; ++h) th_[h] = std::thread([this, h] { run(h); });
    } catch (...) {  // a thread that would not start: release the started ones, then report
      abort_.store(true, std::memory_order_release);
      for (auto& t : th_)
        if (t.joinable()) t.join();
      throw;
    }
  }
  ~ShufflePool() {
    for (auto& t : th_) t.join();
  }
  int64_t batch() const { return B_; }
  uint32_t* slot(int64_t k) {  // js of batch k (job q at + (q % B) * stride), once batch k - R is done
    const int64_t old = k - kSlots;
    if (old >= 0) {
      const int h = (int)(old % kThreads);
      const int64_t need = old / kThreads + 1;
      while (done_[h].v.load(std::memory_order_acquire) < need) std::this_thread::yield();
    }
    return js_.data() + (size_t)((k % kSlots) * B_ * stride_);
  }
  void publish(int64_t k) { filtered_.v.store(k + 1, std::memory_order_release); }

 private:
  static constexpr int kThreads = 2;
  static constexpr int64_t kSlots = 8;
  struct alignas(64) Ctr {
    std::atomic<int64_t> v{0};
  };
  void run(int h) {
    std::vector<int64_t> perm;
    int64_t mine = 0;
    for (int64_t k = h; k < nbatch_; k += kThreads) {
      while (filtered_.v.load(std::memory_order_acquire) <= k) {
        if (abort_.load(std::memory_order_acquire)) return;
        std::this_thread::yield();
      }
      const uint32_t* js = js_.data() + (size_t)((k % kSlots) * B_ * stride_);
      for (int64_t q = k * B_; q < std::min(njobs_, (k + 1) * B_); ++q) {
        const int64_t i = q % n_;
        int32_t* o = out_ + q * b_;
        const int64_t m = rows_[i];
        const int64_t eb = (m == 0) ? 0 : (b_ < m ? b_ : m);
        if (eb > 0) shuffle_prefix(m, eb, js + (size_t)((q - k * B_) * stride_), perm, o);
        for (int64_t c = eb; c < b_; ++c) o[c] = -1;
      }
      done_[h].v.store(++mine, std::memory_order_release);
    }
  }
  const int64_t n_;
  const int64_t* rows_;
  const int64_t b_;
  int32_t* out_;
  const int64_t stride_, njobs_, B_, nbatch_;
  std::vector<uint32_t> js_;
  Ctr filtered_;
  Ctr done_[kThreads];
  std::atomic<bool> abort_{false};
  std::thread th_[kThreads];
};

// The speculative parallel draw for uniform shards (defined below); 1 = not applicable.
static int choice_rounds_parallel(uint32_t key[624], int32_t* pos, int64_t T, int64_t n_workers,
                                  const int64_t* shard_rows, int64_t b, int32_t* out, int64_t max_m);

// The numpy state (key, pos) is written only when a call completes: a call that fails leaves
// it where it was.
static int choice_rounds(uint32_t key[624], int32_t* pos, int64_t T, int64_t n_workers, const int64_t* shard_rows,
                         int64_t b, int32_t* out) {
  if (b < 0) return DOPT_ERR_INVALID;
  if (int rc = check_rounds(key, pos, T, n_workers, shard_rows)) return rc;
  if (T == 0 || n_workers == 0) return DOPT_OK;
  int64_t max_m = 1;
  for (int64_t i = 0; i < n_workers; ++i) max_m = std::max(max_m, shard_rows[i]);
  if (b == 0) return DOPT_OK;  // eb = 0 for every worker: no draw at all (worker.py:21-23)
  if (int rc = choice_rounds_parallel(key, pos, T, n_workers, shard_rows, b, out, max_m); rc != 1) return rc;
  BlockRing ring(key, *pos);
  RingStream st(ring);
  if (max_m > (int64_t(1) << 22)) {  // shards beyond 4M rows: shuffle inline (no 128 MiB js ring)
    std::vector<int64_t> perm;
    std::vector<uint32_t> js((size_t)max_m);
    for (int64_t q = 0; q < T * n_workers; ++q) {
      const int64_t m = shard_rows[q % n_workers];
      const int64_t eb = (m == 0) ? 0 : (b < m ? b : m);
      int32_t* o = out + q * b;
      if (eb > 0) {
        st.draw(m, js.data());
        shuffle_prefix(m, eb, js.data(), perm, o);
      }
      for (int64_t k = eb; k < b; ++k) o[k] = -1;
    }
    st.save(key, pos);
    return DOPT_OK;
  }
  {
    ShufflePool pool(T, n_workers, shard_rows, b, out, max_m);
    const int64_t nj = T * n_workers, B = pool.batch();
    for (int64_t k = 0; k * B < nj; ++k) {
      uint32_t* js = pool.slot(k);
      for (int64_t q = k * B; q < std::min(nj, (k + 1) * B); ++q) {
        const int64_t m = shard_rows[q % n_workers];
        if (m > 0) st.draw(m, js + (q - k * B) * max_m);
      }
      pool.publish(k);
    }
  }  // joins the shuffle threads: out is complete
  st.save(key, pos);
  return DOPT_OK;
}

// ---------------------------------------------------------------------------- parallel advance
// The stream advance of full-shard rounds over UNIFORM shards (every drawing worker has the same
// m >= 2 rows: C3), speculatively in parallel.  The filter is a finite-state machine over the
// word stream: its state before a word is the k of the Fisher-Yates step in progress (m-1 .. 1),
// and two runs that are in the same state before the same word stay together from there on
// (the next word's verdict depends on k alone).  So the stream is cut into segments of kSeg
// blocks, each filtered on a thread of its own from a GUESSED state (k = m - 1; segment 0 from
// the true one), recording the permutation ends it sees, its k before each of its first kWin
// blocks' words and its k at its end.  The stitch (this thread, in segment order) knows the
// true k at a segment's start (the previous segment's end state, true once that segment's run
// had met the true one) and runs the filter from there itself until its k equals the recorded
// k before the same word: from that word on the segment's run IS the true one, so the true
// permutation ends are the stitch's own before it and the segment's after it.  Two runs from
// different states meet after ~1e5 words on average at m = 512 (p90 ~2.6e5, the largest of 60
// samples 4.1e5 words; kWin = 1680 blocks = 1.05M words); a segment whose window holds no
// meeting point is finished by the stitch itself (correct, just sequential).  The words are the
// same whichever thread filters them: a producer thread twists the key from segment start to
// segment start (snapshots), each segment's thread twists and tempers its own blocks.
namespace {

struct ParSeg {
  std::vector<uint16_t> pre;  // k before each word of the segment's first kWin blocks
  std::vector<int64_t> pe;    // word index of the word completing each permutation
  std::vector<uint32_t> vals; // (minibatch draws) every kept word's value, in order
  std::vector<int64_t> cum;   // (minibatch draws) kept words before each block
  uint32_t kend = 0;          // k after the segment's last word
  std::atomic<int64_t> pre_blocks{0};  // blocks of `pre` written so far
  std::atomic<int> done{0};
};

int affinity_cpus() {
  cpu_set_t s;
  if (sched_getaffinity(0, sizeof(s), &s) != 0) return (int)std::thread::hardware_concurrency();
  return CPU_COUNT(&s);
}

int64_t env_i64(const char* name, int64_t dflt) {
  const char* v = getenv(name);
  return v ? atoll(v) : dflt;
}

// the twist and the tempering of a whole block vectorise (x86 function multiversioning: the
// widest of AVX-512 / AVX2 / baseline the host has, picked at load time; sanitizer builds define
// DOPT_NO_MULTIVERSION -- their runtimes are not up yet when the loader runs ifunc resolvers)
#if defined(__x86_64__) && !defined(DOPT_NO_MULTIVERSION)
#define DOPT_MV __attribute__((target_clones("avx512f", "avx2", "default")))
#else
#define DOPT_MV
#endif
DOPT_MV void twist_key(uint32_t* __restrict__ key) {
  int i = 0;
  for (; i < kN - kM; ++i) {
    const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
    key[i] = key[i + kM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
  }
  for (; i < kN - 1; ++i) {
    const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
    key[i] = key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
  }
  const uint32_t y = (key[kN - 1] & kUpper) | (key[0] & kLower);
  key[kN - 1] = key[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
}

DOPT_MV void temper_block(const uint32_t* __restrict__ key, uint32_t* __restrict__ out) {
  for (int k = 0; k < kN; ++k) {
    uint32_t y = key[k];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    out[k] = y;
  }
}

// filter_block that also records k before every word it reads (rec[q] for word q of the block)
inline void filter_block_rec(const uint32_t* out, int32_t& q, uint32_t& k, uint32_t& t, uint32_t* js, uint16_t* rec) {
  while (q < kN && k >= 1) {
    const uint32_t mask = 0xffffffffu >> __builtin_clz(k);
    const uint32_t klo = mask >> 1;
    while (q + 8 <= kN && k - klo >= 8) {
#pragma GCC unroll 8
      for (int u = 0; u < 8; ++u) {
        rec[q + u] = (uint16_t)k;
        const uint32_t v = out[q + u] & mask;
        const uint32_t keep = v <= k;
        js[t] = v;
        t += keep;
        k -= keep;
      }
      q += 8;
    }
    while (q < kN && k > klo) {
      rec[q] = (uint16_t)k;
      const uint32_t v = out[q++] & mask;
      const uint32_t keep = v <= k;
      js[t] = v;
      t += keep;
      k -= keep;
    }
  }
}

class ParAdvance {
 public:
  // keep: also record every kept word's value (the Fisher-Yates j's of minibatch draws; m >= 3,
  // so that every kept word changes k and the recorded k's locate the meeting point in the
  // kept-value stream as well)
  ParAdvance(const uint32_t* key0, int32_t pos0, int64_t m, int64_t perms, int threads, bool keep = false)
      : m_(m), D_((uint32_t)(m - 1)), P_(perms), pos0_(pos0), keep_(keep),
        seg_(std::max<int64_t>(1, env_i64("DOPT_MT_SEG_BLOCKS", 4096))),
        win_(std::max<int64_t>(1, std::min<int64_t>(env_i64("DOPT_MT_WIN_BLOCKS", 1680), seg_))) {
    // expected words per permutation: a draw at k is kept with probability (k + 1) / (mask(k) + 1)
    double wpp = 0.0;
    for (uint32_t k = 1; k <= D_; ++k) wpp += (double)((0xffffffffu >> __builtin_clz(k)) + 1ull) / (double)(k + 1);
    nseg_ = (int64_t)((double)perms * wpp * 1.02 / (double)(seg_ * kN)) + 2;
    key0_.assign(key0, key0 + kN);
    snaps_.resize((size_t)(nseg_ + 1) * kN);
    memcpy(snaps_.data(), key0, sizeof(uint32_t) * kN);
    segs_.reserve((size_t)nseg_);
    for (int64_t j = 0; j < nseg_; ++j) segs_.emplace_back(new ParSeg());
    snap_ready_.store(1, std::memory_order_release);
    ahead_ = std::max<int64_t>(4, 4 * (int64_t)threads);
    try {
      prod_ = std::thread([this] { produce(); });
      for (int h = 0; h < threads; ++h) th_.emplace_back([this] { work(); });
    } catch (...) {
      stop_.store(true, std::memory_order_release);
      join();
      throw;
    }
  }
  ~ParAdvance() {
    stop_.store(true, std::memory_order_release);
    join();
  }
  // The true kept-value stream (keep mode) as pieces (pointer, count) in order: the stitch's own
  // values before each meeting word, then the segment's from there.
  typedef std::pair<const uint32_t*, int64_t> Piece;
  // the stitch; writes numpy's state after the last permutation's last word
  void finish(uint32_t key[kN], int32_t* pos, std::vector<Piece>* pieces = nullptr) {
    int64_t done = 0, last = -1;
    uint32_t ktrue = D_;  // the true k before the current segment's first word
    std::vector<uint32_t> kk(kN), out(kN), js((size_t)m_);
    std::vector<uint16_t> rec(kN);
    auto trans = [](const uint16_t* r, int32_t n) {  // kept words among the first n (k changes on each)
      int64_t c = 0;
      for (int32_t x = 0; x < n; ++x) c += r[x + 1] != r[x];
      return c;
    };
    for (int64_t j = 0; last < 0; ++j) {
      const int64_t b0 = j * seg_, b1 = b0 + seg_;
      ParSeg* s = j < nseg_ ? segs_[(size_t)j].get() : nullptr;
      if (j == 0) {  // segment 0 ran from the true state
        while (!s->done.load(std::memory_order_acquire)) std::this_thread::yield();
        if (keep_) pieces->emplace_back(s->vals.data(), s->cum[(size_t)seg_]);
        for (int64_t e : s->pe)
          if (++done == P_) {
            last = e;
            break;
          }
        ktrue = s->kend;
        release(j);
        continue;
      }
      // from the true state until it meets the segment's recorded run (or to the segment's end),
      // a block at a time: the recording filter, then the first word where the two k agree
      key_of_block(b0, kk.data());
      uint32_t k = ktrue, t = 0;
      bool met = false;
      int64_t meet = 0, seg_at = 0;  // keep: the segment's kept words before the meeting word
      std::vector<int64_t> ends;
      std::vector<uint32_t>* own = nullptr;  // keep: the stitch's own kept values in this segment
      if (keep_) {
        owns_.emplace_back(new std::vector<uint32_t>());
        own = owns_.back().get();
      }
      for (int64_t b = b0; b < b1 && !met && last < 0; ++b) {
        if (b != b0) twist_key(kk.data());
        temper_block(kk.data(), out.data());
        ends.clear();
        const int64_t tb = keep_ ? (int64_t)own->size() : 0;  // kept before this block
        if (keep_) own->resize((size_t)(tb + kN + 1));
        uint32_t* jsb = keep_ ? own->data() + tb : js.data();
        uint32_t tk = 0;
        for (int32_t q = 0; q < kN;) {
          filter_block_rec(out.data(), q, k, keep_ ? tk : t, jsb, rec.data());
          if (k == 0) {
            ends.push_back(b * kN + q - 1);
            k = D_;
            t = 0;
          }
        }
        int32_t qm = kN;
        const uint16_t* pre = nullptr;
        if (s && b < b0 + win_) {
          while (s->pre_blocks.load(std::memory_order_acquire) <= b - b0) std::this_thread::yield();
          pre = s->pre.data() + (b - b0) * kN;
          for (int32_t x = 0; x < kN; ++x)
            if (rec[(size_t)x] == pre[x]) {
              qm = x;
              break;
            }
        }
        if (keep_) {  // keep the stitch's values up to the meeting word (all of the block without one)
          own->resize((size_t)(tb + (qm < kN ? trans(rec.data(), qm) : (int64_t)tk)));
          if (qm < kN) {
            while (!s->done.load(std::memory_order_acquire)) std::this_thread::yield();  // s->cum
            seg_at = s->cum[(size_t)(b - b0)] + trans(pre, qm);
          }
        }
        for (int64_t e : ends)
          if (e < b * kN + qm && ++done == P_) {
            last = e;
            break;
          }
        if (qm < kN) {
          met = true;
          meet = b * kN + qm;
        }
      }
      if (met)
        while (!s->done.load(std::memory_order_acquire)) std::this_thread::yield();
      if (keep_) {
        pieces->emplace_back(own->data(), (int64_t)own->size());
        if (met) pieces->emplace_back(s->vals.data() + seg_at, s->cum[(size_t)seg_] - seg_at);
      }
      if (last >= 0) break;
      if (!met) {  // no meeting point (or a segment past the planned ones): the stitch's run is the truth
        ktrue = k;
        release(j);
        continue;
      }
      for (int64_t e : s->pe)
        if (e >= meet && ++done == P_) {
          last = e;
          break;
        }
      ktrue = s->kend;
      release(j);
    }
    stop_.store(true, std::memory_order_release);
    // numpy's state: the key of the block holding the last word, pos just past it (1 .. 624)
    const int64_t blk = last / kN;
    *pos = (int32_t)(last - blk * kN + 1);
    key_of_block(blk, key);
  }

 private:
  int64_t snap_count() const { return snap_ready_.load(std::memory_order_acquire); }
  void produce() {
    std::vector<uint32_t> k(key0_);
    for (int64_t j = 1; j <= nseg_; ++j) {
      for (int64_t b = 0; b < seg_; ++b) {
        if (stop_.load(std::memory_order_relaxed)) return;
        twist_key(k.data());
      }
      memcpy(snaps_.data() + (size_t)j * kN, k.data(), sizeof(uint32_t) * kN);
      snap_ready_.store(j + 1, std::memory_order_release);
    }
  }
  // the key of block b: from the nearest snapshot (waiting for the producer), twisted on
  void key_of_block(int64_t b, uint32_t* key) {
    const int64_t j = std::min(b / seg_, nseg_);
    while (snap_count() <= j) std::this_thread::yield();  // the producer runs until stop_
    memcpy(key, snaps_.data() + (size_t)j * kN, sizeof(uint32_t) * kN);
    for (int64_t x = j * seg_; x < b; ++x) twist_key(key);
  }
  // Segment j is stitched: its k records and permutation ends are dead (its kept values stay while
  // pieces point into them), and the filter threads may run that much further ahead.
  void release(int64_t j) {
    if (j < nseg_) {
      ParSeg& s = *segs_[(size_t)j];
      while (!s.done.load(std::memory_order_acquire) && j > 0 && !stop_.load(std::memory_order_acquire)) {
        // a segment the stitch finished itself may still be filtering: its thread owns the buffers
        std::this_thread::yield();
      }
      std::vector<uint16_t>().swap(s.pre);
      std::vector<int64_t>().swap(s.pe);
    }
    stitched_.store(j + 1, std::memory_order_release);
  }
  void work() {
    for (;;) {
      const int64_t j = next_.fetch_add(1);
      if (j >= nseg_) return;
      // bounded run-ahead: at most ahead_ segments past the stitch hold their buffers
      while (j >= stitched_.load(std::memory_order_acquire) + ahead_) {
        if (stop_.load(std::memory_order_acquire)) return;
        std::this_thread::yield();
      }
      while (snap_count() <= j) {
        if (stop_.load(std::memory_order_acquire)) return;
        std::this_thread::yield();
      }
      ParSeg& s = *segs_[(size_t)j];
      if (!run_segment(j, s)) return;
      s.done.store(1, std::memory_order_release);
    }
  }
  // Filter segment j (blocks [j seg, (j + 1) seg)) from k = m - 1 (segment 0: the call's start
  // state, word pos0 of block 0); records pe, kend and (j > 0) k before each word of the first
  // win blocks.
  bool run_segment(int64_t j, ParSeg& s) {
    const int64_t b0 = j * seg_, b1 = b0 + seg_;
    std::vector<uint32_t> key(snaps_.begin() + j * kN, snaps_.begin() + (j + 1) * kN), out(kN), js((size_t)m_);
    s.pe.clear();
    s.pre.assign(j > 0 ? (size_t)(win_ * kN) : 0, 0);
    if (keep_) {  // one index t over the whole segment: js[t] is the next kept word's slot
      s.vals.resize((size_t)(seg_ * kN + 1));
      s.cum.assign((size_t)(seg_ + 1), 0);
    }
    uint32_t* jsp = keep_ ? s.vals.data() : js.data();
    uint32_t k = D_, t = 0;
    for (int64_t b = b0; b < b1; ++b) {
      if (b != b0) twist_key(key.data());  // the snapshot is block b0's key
      temper_block(key.data(), out.data());
      if (keep_) s.cum[(size_t)(b - b0)] = t;
      int32_t q = (b == 0) ? pos0_ : 0;
      uint16_t* rec = (j > 0 && b < b0 + win_) ? s.pre.data() + (b - b0) * kN : nullptr;
      while (q < kN) {
        if (rec) filter_block_rec(out.data(), q, k, t, jsp, rec);
        else filter_block(out.data(), q, k, t, jsp);
        if (k == 0) {
          s.pe.push_back(b * kN + q - 1);
          k = D_;
          if (!keep_) t = 0;
        }
      }
      if (rec) s.pre_blocks.store(b - b0 + 1, std::memory_order_release);
      if ((b & 255) == 0 && stop_.load(std::memory_order_relaxed)) return false;
    }
    s.kend = k;
    if (keep_) s.cum[(size_t)seg_] = t;
    return true;
  }
  void join() {
    for (auto& t : th_)
      if (t.joinable()) t.join();
    if (prod_.joinable()) prod_.join();
  }

  const int64_t m_;
  const uint32_t D_;
  const int64_t P_;
  const int32_t pos0_;
  const bool keep_;
  const int64_t seg_, win_;
  int64_t nseg_;
  std::vector<std::unique_ptr<std::vector<uint32_t>>> owns_;  // the stitch's kept values (pieces point in)
  std::vector<uint32_t> key0_, snaps_;
  std::vector<std::unique_ptr<ParSeg>> segs_;
  std::atomic<int64_t> snap_ready_{0}, next_{0}, stitched_{0};
  int64_t ahead_ = 8;  // segments the filter threads may run past the stitch (set from the thread count)
  std::atomic<bool> stop_{false};
  std::thread prod_;
  std::vector<std::thread> th_;
};

}  // namespace

namespace {
// Uniform shards (every drawing worker has m rows, the rest 0 / 1 -- they draw nothing): the
// number of drawing workers, or -1.  min_m: 2 for the advance, 3 for minibatch draws (keep mode).
int64_t uniform_drawing(int64_t n_workers, const int64_t* rows, int64_t max_m, int64_t min_m) {
  if (max_m < min_m || max_m > 4096) return -1;
  int64_t drawing = 0;
  for (int64_t i = 0; i < n_workers; ++i) {
    if (rows[i] > 1 && rows[i] != max_m) return -1;
    drawing += rows[i] == max_m;
  }
  return drawing;
}

// filter threads: min(12, the rank's CPUs - 4), the CPUs split over the ranks of this node when
// every rank sees them all (torchrun: LOCAL_WORLD_SIZE ranks, one affinity set)
int par_threads() {
  const int64_t local = std::max<int64_t>(1, env_i64("LOCAL_WORLD_SIZE", 1));
  const int64_t cpus = affinity_cpus() / local;
  return (int)env_i64("DOPT_MT_THREADS", std::min<int64_t>(12, std::max<int64_t>(0, cpus - 4)));
}

bool par_worth(int64_t T, int64_t drawing, int64_t m) {  // >= 3 segments of words
  return (double)T * drawing * (m - 1) * 1.38 >= 3.0 * (double)(env_i64("DOPT_MT_SEG_BLOCKS", 4096) * kN);
}
}  // namespace

static int choice_rounds_parallel_part(uint32_t key[624], int32_t* pos, int64_t T, int64_t n, const int64_t* rows,
                                       int64_t b, int32_t* out, int64_t max_m, int64_t drawing, int threads);

// Minibatch draws over many rounds: the parallel filter keeps every kept word's value until the
// shuffles have read them (~4 bytes per word, ~705 words per permutation of 512), so the rounds go
// in parts of at most kKeepSegs segments of words each (~330 MB of values per part).
constexpr int64_t kKeepSegs = 32;
static int choice_rounds_parallel(uint32_t key[624], int32_t* pos, int64_t T, int64_t n, const int64_t* rows,
                                  int64_t b, int32_t* out, int64_t max_m) {
  const int64_t drawing = uniform_drawing(n, rows, max_m, 3);
  const int threads = par_threads();
  if (drawing <= 0 || threads < 2 || !par_worth(T, drawing, max_m)) return 1;
  const double words_per_round = (double)drawing * (double)(max_m - 1) * 1.38;
  const double cap_words = (double)kKeepSegs * (double)env_i64("DOPT_MT_SEG_BLOCKS", 4096) * kN;
  const int64_t per = std::max<int64_t>(1, (int64_t)(cap_words / std::max(1.0, words_per_round)));
  uint32_t kl[kN];  // the state advances part by part; numpy's copy only when every part is done
  int32_t pl = *pos;
  memcpy(kl, key, sizeof(kl));
  for (int64_t t0 = 0; t0 < T;) {
    int64_t tp = std::min(per, T - t0);
    if (T - t0 - tp > 0 && !par_worth(T - t0 - tp, drawing, max_m)) tp = T - t0;  // no short tail part
    // (every part is long enough: per rounds hold kKeepSegs segments of words, a merged tail more)
    const int rc = choice_rounds_parallel_part(kl, &pl, tp, n, rows, b, out + t0 * n * b, max_m, drawing, threads);
    if (rc) return rc;
    t0 += tp;
  }
  memcpy(key, kl, sizeof(kl));
  *pos = pl;
  return DOPT_OK;
}

static int choice_rounds_parallel_part(uint32_t key[624], int32_t* pos, int64_t T, int64_t n, const int64_t* rows,
                                       int64_t b, int32_t* out, int64_t max_m, int64_t drawing, int threads) {
  if (T <= 0) return DOPT_OK;
  uint32_t key1[kN];
  int32_t pos1 = *pos;
  memcpy(key1, key, sizeof(key1));
  ParAdvance par(key1, pos1, max_m, T * drawing, threads, true);
  std::vector<ParAdvance::Piece> pieces;
  par.finish(key1, &pos1, &pieces);
  std::vector<int64_t> ps(pieces.size() + 1, 0);  // stream offset of each piece
  for (size_t x = 0; x < pieces.size(); ++x) ps[x + 1] = ps[x] + pieces[x].second;
  const int64_t D = max_m - 1;
  if (ps.back() < T * drawing * D) return DOPT_ERR_RUNTIME;  // (the stitch ran to the P-th end)
  std::vector<int64_t> rank((size_t)n, -1);
  for (int64_t i = 0, r = 0; i < n; ++i)
    if (rows[i] == max_m) rank[(size_t)i] = r++;
  // the Fisher-Yates shuffles: jobs (round, worker) in contiguous ranges over the threads
  const int64_t nj = T * n;
  std::atomic<bool> fail{false};
  auto body = [&](int64_t q0, int64_t q1) {
    std::vector<int64_t> perm;
    std::vector<uint32_t> js((size_t)max_m);
    for (int64_t q = q0; q < q1; ++q) {
      const int64_t t = q / n, i = q % n, m = rows[i];
      const int64_t eb = (m == 0) ? 0 : (b < m ? b : m);
      int32_t* o = out + q * b;
      if (m == max_m) {  // gather the permutation's D kept values from the pieces
        int64_t off = (t * drawing + rank[(size_t)i]) * D, got = 0;
        size_t x = (size_t)(std::upper_bound(ps.begin(), ps.end(), off) - ps.begin()) - 1;
        while (got < D) {
          const int64_t in = off - ps[x], take = std::min(D - got, pieces[x].second - in);
          memcpy(js.data() + got, pieces[x].first + in, (size_t)take * sizeof(uint32_t));
          got += take;
          off += take;
          ++x;
        }
      }
      if (eb > 0) shuffle_prefix(m, eb, js.data(), perm, o);  // m = 1: [0] without a draw
      for (int64_t c = eb; c < b; ++c) o[c] = -1;
    }
  };
  {
    std::vector<std::thread> th;
    const int64_t per = (nj + threads - 1) / threads;
    try {
      for (int h = 1; h < threads && h * per < nj; ++h) th.emplace_back(body, h * per, std::min(nj, (h + 1) * per));
    } catch (...) {
      fail.store(true);
    }
    body(0, std::min(nj, per));
    for (auto& x : th) x.join();
    if (fail.load()) {  // a thread that would not start: its range here
      for (int h = 1 + (int)th.size(); h < threads && h * per < nj; ++h) body(h * per, std::min(nj, (h + 1) * per));
    }
  }
  memcpy(key, key1, sizeof(key1));
  *pos = pos1;
  return DOPT_OK;
}

static int advance_rounds(uint32_t key[624], int32_t* pos, int64_t T, int64_t n_workers, const int64_t* shard_rows) {
  if (int rc = check_rounds(key, pos, T, n_workers, shard_rows)) return rc;
  if (T == 0 || n_workers == 0) return DOPT_OK;
  int64_t max_m = 1;
  for (int64_t i = 0; i < n_workers; ++i) max_m = std::max(max_m, shard_rows[i]);
  // uniform shards (every drawing worker has m rows, the rest 0 / 1) and a long enough stream:
  // the speculative parallel filter (DOPT_MT_THREADS: filter threads, 0 / 1 = this thread only)
  const int64_t drawing = uniform_drawing(n_workers, shard_rows, max_m, 2);
  const int threads = par_threads();
  if (drawing > 0 && threads >= 2 && par_worth(T, drawing, max_m)) {
    ParAdvance par(key, *pos, max_m, T * drawing, threads);
    par.finish(key, pos);
    return DOPT_OK;
  }
  BlockRing ring(key, *pos);
  RingStream st(ring);
  // the recording filter into a scratch row (an L1-resident store per word is cheaper than the
  // branchy code the compiler makes of the counting-only form: 2.7 vs 3.2 ns per draw)
  std::vector<uint32_t> js((size_t)max_m);
  for (int64_t t = 0; t < T; ++t)
    for (int64_t i = 0; i < n_workers; ++i)
      if (shard_rows[i] > 0) st.draw(shard_rows[i], js.data());  // every choice() is a whole permutation
  st.save(key, pos);
  return DOPT_OK;
}

// Host threads or buffers that cannot be had (std::system_error / std::bad_alloc) come back as
// error codes, not as exceptions through the C ABI.
extern "C" int dopt_mt_choice_rounds(uint32_t key[624], int32_t* pos, int64_t T, int64_t n_workers,
                                     const int64_t* shard_rows, int64_t b, int32_t* out) {
  try {
    return choice_rounds(key, pos, T, n_workers, shard_rows, b, out);
  } catch (const std::bad_alloc&) {
    return DOPT_ERR_NOMEM;
  } catch (...) {
    return DOPT_ERR_RUNTIME;
  }
}

extern "C" int dopt_mt_advance_rounds(uint32_t key[624], int32_t* pos, int64_t T, int64_t n_workers,
                                      const int64_t* shard_rows) {
  try {
    return advance_rounds(key, pos, T, n_workers, shard_rows);
  } catch (const std::bad_alloc&) {
    return DOPT_ERR_NOMEM;
  } catch (...) {
    return DOPT_ERR_RUNTIME;
  }
}
