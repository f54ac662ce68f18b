// Native pre-tokenised token loader (C ABI, loaded with ctypes by nanodiloco_amd/data/memmap.py).
//
// The reference tokenises the whole dataset on every rank at start-up and pads batches on the
// training thread (REF/nanodiloco/training_utils/utils.py:45-55, REF/nanodiloco/main.py:79-96,
// num_workers=0).  Here the corpus is pre-tokenised once into flat little-endian uint16/uint32
// shard files; this loader memory-maps them (no copy, no parse), cuts fixed seq_len windows, gives
// rank r the windows r, r+W, r+2W, ... (disjoint across DiLoCo workers), shuffles them per epoch
// with a seeded Fisher-Yates permutation, and assembles int64 batches on a background thread into
// a ring of caller-owned (pinned) host buffers.  The stream is a pure function of
// (seed, rank, world, cursor), so checkpoints resume exactly.
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

struct Loader {
  std::vector<Shard> shards;
  int token_bytes = 2;
  int64_t seq_len = 0, batch = 0;
  uint64_t seed = 0;
  int rank = 0, world = 1;
  bool shuffle = true;
  int64_t my_windows = 0;        // windows owned by this rank per epoch
  std::vector<int64_t> perm;     // permutation of [0, my_windows) for the current epoch
  int64_t perm_epoch = -1;
  int64_t cursor = 0;            // samples handed out so far (monotonic across epochs)

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

  void build_perm(int64_t epoch) {
    perm.resize(my_windows);
    for (int64_t i = 0; i < my_windows; ++i) perm[i] = i;
    if (shuffle) {
      uint64_t s = seed ^ (0xA24BAED4963EE407ull * (uint64_t)(epoch + 1)) ^ (0x9FB21C651E98DF25ull * (uint64_t)(rank + 1));
      for (int64_t i = my_windows - 1; i > 0; --i) {
        int64_t j = (int64_t)(splitmix64(s) % (uint64_t)(i + 1));
        std::swap(perm[i], perm[j]);
      }
    }
    perm_epoch = epoch;
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
    for (int64_t b = 0; b < batch; ++b) {
      int64_t sample = cur + b;
      int64_t epoch = sample / my_windows;
      int64_t idx = sample % my_windows;
      if (epoch != perm_epoch) build_perm(epoch);
      int64_t local = perm[idx];
      int64_t gw = local * world + rank;
      read_window(gw, out + b * seq_len);
    }
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
  L->my_windows = gw / world;  // equal count per rank (drop_last semantics)
  if (L->my_windows <= 0) { snprintf(err, errlen, "dataset too small: %lld windows for %d ranks", (long long)gw, world); delete L; return nullptr; }
  L->nslots = nslots;
  L->slots.assign(slot_ptrs, slot_ptrs + nslots);
  L->state.assign(nslots, 0);
  L->start();
  return L;
}

int64_t nd_loader_windows_per_rank(void* h) { return static_cast<Loader*>(h)->my_windows; }

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

void nd_loader_destroy(void* h) { delete static_cast<Loader*>(h); }

}  // extern "C"
