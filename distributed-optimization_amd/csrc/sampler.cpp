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

#include <algorithm>
#include <atomic>
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

// The numpy state (key, pos) is written only when a call completes: a call that fails leaves
// it where it was.
static int choice_rounds(uint32_t key[624], int32_t* pos, int64_t T, int64_t n_workers, const int64_t* shard_rows,
                         int64_t b, int32_t* out) {
  if (b < 0) return DOPT_ERR_INVALID;
  if (int rc = check_rounds(key, pos, T, n_workers, shard_rows)) return rc;
  if (T == 0 || n_workers == 0) return DOPT_OK;
  int64_t max_m = 1;
  for (int64_t i = 0; i < n_workers; ++i) max_m = std::max(max_m, shard_rows[i]);
  BlockRing ring(key, *pos);
  RingStream st(ring);
  if (b == 0) {  // eb = 0 for every worker: no draw at all (worker.py:21-23)
    st.save(key, pos);
    return DOPT_OK;
  }
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

static int advance_rounds(uint32_t key[624], int32_t* pos, int64_t T, int64_t n_workers, const int64_t* shard_rows) {
  if (int rc = check_rounds(key, pos, T, n_workers, shard_rows)) return rc;
  if (T == 0 || n_workers == 0) return DOPT_OK;
  BlockRing ring(key, *pos);
  RingStream st(ring);
  int64_t max_m = 1;
  for (int64_t i = 0; i < n_workers; ++i) max_m = std::max(max_m, shard_rows[i]);
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
