// Native pre-tokenised token loader (C ABI, loaded with ctypes by nanodiloco_amd/data/memmap.py).
//
// The reference tokenises the whole dataset on every rank at start-up and pads batches on the
// training thread (REF/nanodiloco/training_utils/utils.py:45-55, REF/nanodiloco/main.py:79-96,
// num_workers=0).  Here the corpus is pre-tokenised once into flat little-endian uint16/uint32
// shard files; this loader memory-maps them (no copy, no parse), cuts fixed seq_len windows and
// assembles int64 batches on a background thread into a ring of caller-owned (pinned) host buffers.
//
// Sample order: ONE global stream of window positions q = 0, 1, 2, ... (epoch q / G, G = total
// windows; window = perm_epoch(q mod G), a seeded Feistel permutation with cycle walking -- O(1)
// memory, any G).  Rank r of W takes positions base + r, base + r + W, base + r + 2W, ...: the DiLoCo
// workers' streams are disjoint inside every epoch and together consume the global stream in order.
// The state is (base, W, cursor); all workers advance in lockstep, so the global position reached is
// base + cursor * W.  An elastic resume on W' workers (utils/checkpoint.py) restarts every worker, old
// and new, at base' = that position: no window is repeated and none skipped across the resize.
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <fcntl.h>
#include <mutex>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

namespace {

struct Shard {
  const uint8_t* base = nullptr;
  size_t bytes = 0;
  int64_t tokens = 0;
  int64_t first_window = 0;  // global window index of this shard's first window
  int64_t windows = 0;
};

inline uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Bijection of [0, n) keyed by (seed, epoch): a 4-round balanced Feistel network on the smallest even
// bit width covering n, with cycle walking (values >= n are permuted again; fewer than 4 steps expected).
struct Perm {
  uint64_t n = 1, mask = 1, key[4] = {0, 0, 0, 0};
  int half = 1;
  void init(uint64_t n_, uint64_t seed, uint64_t epoch) {
    n = n_;
    int bits = 2;
    while (bits < 64 && (1ull << bits) < n) ++bits;
    half = (bits + 1) / 2;
    mask = (1ull << half) - 1;
    uint64_t s = seed ^ (0xA24BAED4963EE407ull * (epoch + 1));
    for (auto& k : key) k = splitmix64(s);
  }
  uint64_t once(uint64_t x) const {
    uint64_t l = x >> half, r = x & mask;
    for (int i = 0; i < 4; ++i) {
      uint64_t h = r ^ key[i];
      h = (h ^ (h >> 31)) * 0x7FB5D329728EA185ull;
      h = (h ^ (h >> 27)) * 0x81DADEF4BC2DD44Dull;
      const uint64_t nl = r, nr = (l ^ (h ^ (h >> 33))) & mask;
      l = nl;
      r = nr;
    }
    return (l << half) | r;
  }
  uint64_t operator()(uint64_t x) const {
    do x = once(x);
    while (x >= n);
    return x;
  }
};

struct Loader {
  std::vector<Shard> shards;
  int token_bytes = 2;
  int64_t seq_len = 0, batch = 0;
  uint64_t seed = 0;
  int rank = 0, world = 1;
  bool shuffle = true;
  int64_t total_windows = 0;     // G: windows of the corpus, one epoch of the global stream
  int64_t base = 0;              // global stream position this rank's cursor counts from
  Perm perm;                     // window order of epoch perm_epoch
  int64_t perm_epoch = -1;
  int64_t cursor = 0;            // samples handed out since `base` (monotonic across epochs)

  // prefetch ring
  int nslots = 0;
  std::vector<int64_t*> slots;
  std::vector<int> state;        // 0 empty, 1 full
  int64_t produce_idx = 0, consume_idx = 0;
  int64_t produce_cursor = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::thread worker;
  std::atomic<bool> stop{false};

  ~Loader() {
    stop_worker();
    for (auto& s : shards)
      if (s.base) munmap(const_cast<uint8_t*>(s.base), s.bytes);
  }

  void stop_worker() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    if (worker.joinable()) worker.join();
  }

  // global window of this rank's sample `sample` (counted from `base`); `pc` / `pe`: the caller's
  // cached permutation and its epoch (the worker thread's own, or a local one)
  int64_t window_of(int64_t sample, Perm& pc, int64_t& pe) const {
    const int64_t q = base + rank + sample * (int64_t)world;
    const int64_t epoch = q / total_windows, idx = q % total_windows;
    if (!shuffle) return idx;
    if (epoch != pe) {
      pc.init((uint64_t)total_windows, seed, (uint64_t)epoch);
      pe = epoch;
    }
    return (int64_t)pc((uint64_t)idx);
  }

  void read_window(int64_t gw, int64_t* out) const {
    // locate shard (few shards: linear scan is fine)
    const Shard* sh = nullptr;
    for (const auto& s : shards)
      if (gw >= s.first_window && gw < s.first_window + s.windows) { sh = &s; break; }
    int64_t off = (gw - sh->first_window) * seq_len;
    if (token_bytes == 2) {
      const uint16_t* p = reinterpret_cast<const uint16_t*>(sh->base) + off;
      for (int64_t t = 0; t < seq_len; ++t) out[t] = p[t];
    } else {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(sh->base) + off;
      for (int64_t t = 0; t < seq_len; ++t) out[t] = p[t];
    }
  }

  // Fill `out` (batch*seq_len int64) with the samples starting at sample index `cur`.
  void fill(int64_t cur, int64_t* out) {
    for (int64_t b = 0; b < batch; ++b) read_window(window_of(cur + b, perm, perm_epoch), out + b * seq_len);
  }

  void run() {
    for (;;) {
      int slot;
      int64_t cur;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop.load() || state[produce_idx % nslots] == 0; });
        if (stop) return;
        slot = (int)(produce_idx % nslots);
        cur = produce_cursor;
      }
      fill(cur, slots[slot]);
      {
        std::lock_guard<std::mutex> g(mu);
        state[slot] = 1;
        produce_idx++;
        produce_cursor = cur + batch;
      }
      cv.notify_all();
    }
  }

  void start() {
    stop = false;
    std::fill(state.begin(), state.end(), 0);
    produce_idx = consume_idx = 0;
    produce_cursor = cursor;
    worker = std::thread([this] { run(); });
  }
};

}  // namespace

extern "C" {

// paths: newline-separated list of shard files.  Returns nullptr on error (message in err).
void* nd_loader_create(const char* paths, int token_bytes, int64_t seq_len, int64_t batch, uint64_t seed, int rank,
                       int world, int shuffle, int nslots, int64_t** slot_ptrs, char* err, int errlen) {
  auto* L = new Loader();
  L->token_bytes = token_bytes;
  L->seq_len = seq_len;
  L->batch = batch;
  L->seed = seed;
  L->rank = rank;
  L->world = world;
  L->shuffle = shuffle != 0;
  std::string all(paths);
  size_t pos = 0;
  int64_t gw = 0;
  while (pos <= all.size()) {
    size_t nl = all.find('\n', pos);
    std::string p = all.substr(pos, nl == std::string::npos ? std::string::npos : nl - pos);
    pos = (nl == std::string::npos) ? all.size() + 1 : nl + 1;
    if (p.empty()) continue;
    int fd = open(p.c_str(), O_RDONLY);
    if (fd < 0) { snprintf(err, errlen, "cannot open %s", p.c_str()); delete L; return nullptr; }
    struct stat st;
    fstat(fd, &st);
    Shard s;
    s.bytes = (size_t)st.st_size;
    s.tokens = (int64_t)(s.bytes / token_bytes);
    s.windows = s.tokens / seq_len;
    s.first_window = gw;
    if (s.bytes > 0) {
      void* m = mmap(nullptr, s.bytes, PROT_READ, MAP_PRIVATE, fd, 0);
      if (m == MAP_FAILED) { close(fd); snprintf(err, errlen, "mmap failed %s", p.c_str()); delete L; return nullptr; }
      madvise(m, s.bytes, MADV_RANDOM);
      s.base = (const uint8_t*)m;
    }
    close(fd);
    gw += s.windows;
    L->shards.push_back(s);
  }
  L->total_windows = gw;
  if (gw < world) { snprintf(err, errlen, "dataset too small: %lld windows for %d ranks", (long long)gw, world); delete L; return nullptr; }
  L->nslots = nslots;
  L->slots.assign(slot_ptrs, slot_ptrs + nslots);
  L->state.assign(nslots, 0);
  L->start();
  return L;
}

// windows this rank reads per epoch of the global stream (floor; one rank may read one more)
int64_t nd_loader_windows_per_rank(void* h) {
  auto* L = static_cast<Loader*>(h);
  return L->total_windows / L->world;
}

int64_t nd_loader_total_windows(void* h) { return static_cast<Loader*>(h)->total_windows; }

// global stream position this rank's cursor counts from, and (setter) restart from `base`, cursor 0
int64_t nd_loader_base(void* h) { return static_cast<Loader*>(h)->base; }

// which global window this rank's sample `sample` (counted from base) reads (tests, diagnostics)
int64_t nd_loader_window_of(void* h, int64_t sample) {
  auto* L = static_cast<Loader*>(h);
  Perm pc;  // the worker thread owns L->perm
  int64_t pe = -1;
  return L->window_of(sample, pc, pe);
}

// Blocks until the next batch is ready; returns its slot index (caller reads slot buffer, then
// calls nd_loader_release(slot)).
int nd_loader_next(void* h) {
  auto* L = static_cast<Loader*>(h);
  std::unique_lock<std::mutex> lk(L->mu);
  int slot = (int)(L->consume_idx % L->nslots);
  L->cv.wait(lk, [&] { return L->state[slot] == 1; });
  L->consume_idx++;
  L->cursor += L->batch;
  return slot;
}

void nd_loader_release(void* h, int slot) {
  auto* L = static_cast<Loader*>(h);
  {
    std::lock_guard<std::mutex> g(L->mu);
    L->state[slot] = 0;
  }
  L->cv.notify_all();
}

int64_t nd_loader_cursor(void* h) { return static_cast<Loader*>(h)->cursor; }

void nd_loader_seek(void* h, int64_t cursor) {
  auto* L = static_cast<Loader*>(h);
  L->stop_worker();
  L->cursor = cursor;
  L->start();
}

void nd_loader_set_base(void* h, int64_t base, int64_t cursor) {
  auto* L = static_cast<Loader*>(h);
  L->stop_worker();
  L->base = base;
  L->cursor = cursor;
  L->start();
}

void nd_loader_destroy(void* h) { delete static_cast<Loader*>(h); }

}  // extern "C"
