// Host-side sanitizer test of the native token loader (built with -fsanitize=address,undefined by
// tests/test_native_sanitize.py; GPU sanitizers are not available on the MI355X pool).
// Exercises create / next / release / seek / destroy across epochs with several ring depths.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

extern "C" {
void* nd_loader_create(const char* paths, int token_bytes, int64_t seq_len, int64_t batch, uint64_t seed, int rank,
                       int world, int shuffle, int nslots, int64_t** slot_ptrs, char* err, int errlen);
int nd_loader_next(void* h);
void nd_loader_release(void* h, int slot);
int64_t nd_loader_cursor(void* h);
void nd_loader_seek(void* h, int64_t cursor);
void nd_loader_destroy(void* h);
int64_t nd_loader_windows_per_rank(void* h);
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const char* path = argv[1];
  const int T = 16, B = 3;
  for (int nslots = 1; nslots <= 4; ++nslots) {
    std::vector<std::vector<int64_t>> bufs(nslots, std::vector<int64_t>(B * T));
    std::vector<int64_t*> ptrs(nslots);
    for (int i = 0; i < nslots; ++i) ptrs[i] = bufs[i].data();
    char err[256];
    void* h = nd_loader_create(path, 2, T, B, 7, 1, 2, 1, nslots, ptrs.data(), err, 256);
    if (!h) { fprintf(stderr, "create failed: %s\n", err); return 1; }
    const int64_t w = nd_loader_windows_per_rank(h);
    std::vector<int64_t> first;
    for (int it = 0; it < 3 * (int)(w / B + 1); ++it) {  // several epochs
      int s = nd_loader_next(h);
      for (int b = 0; b < B; ++b)
        for (int t = 1; t < T; ++t)
          if (bufs[s][b * T + t] != bufs[s][b * T + t - 1] + 1) { fprintf(stderr, "non-contiguous window\n"); return 1; }
      if (it == 5) first.assign(bufs[s].begin(), bufs[s].end());
      nd_loader_release(h, s);
    }
    nd_loader_seek(h, 5 * B);
    int s = nd_loader_next(h);
    if (memcmp(first.data(), bufs[s].data(), first.size() * sizeof(int64_t)) != 0) { fprintf(stderr, "seek mismatch\n"); return 1; }
    nd_loader_release(h, s);
    nd_loader_destroy(h);
  }
  printf("ok\n");
  return 0;
}
