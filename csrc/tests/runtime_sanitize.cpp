// Host-side sanitizer driver for csrc/runtime/runtime.cpp (SURVEY.md §5 "race detection /
// sanitizers": ASan + UBSan debug build of the native runtime). Built and run by
// tests/test_runtime_sanitize_cpu.py as  g++ -fsanitize=address,undefined runtime.cpp this.cpp.
// Exercises every exported entry point over a sweep of shapes, including the cap-too-small and
// malformed-input paths, and checks the invariants the Python side relies on.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" {
int ddl_sched_build(int kind, int n_stages, int n_micro, int32_t* out, int cap);
int ddl_sched_verify(const int32_t* acts, int n, int n_stages);
int ddl_plan_epoch(const int32_t* idx, int G, int count, int batch, const uint64_t* seeds, int shuffle,
                   int32_t* out);
int ddl_bucket_plan(const int64_t* sizes, int n, int64_t cap_bytes, int elem_bytes, int32_t* out);
int ddl_markov_walk(const int64_t* next_tok, const double* cum, int br, const int64_t* cur0, const double* U,
                    int B, int S, int64_t bos, int64_t* out);
int ddl_runtime_version();
}

static int failures = 0;
#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                         \
    }                                                                     \
  } while (0)

static void schedules() {
  for (int kind = 0; kind < 3; ++kind)
    for (int S = 1; S <= 8; ++S)
      for (int M = 1; M <= 12; ++M) {
        const int need = -ddl_sched_build(kind, S, M, nullptr, 0);
        CHECK(need > 0);
        std::vector<int32_t> acts((size_t)need * 5);  // exact size: ASan flags any overrun
        CHECK(ddl_sched_build(kind, S, M, acts.data(), need) == need);
        CHECK(ddl_sched_verify(acts.data(), need, S) == 0);
        if (S > 1) {  // break one receive's micro-batch id: the verifier must notice
          for (int i = 0; i < need; ++i)
            if (acts[5 * i + 1] >= 2 && acts[5 * i + 3] >= 0 && M > 1) {
              std::vector<int32_t> bad = acts;
              bad[5 * i + 2] = (bad[5 * i + 2] + 1) % M;
              CHECK(ddl_sched_verify(bad.data(), need, S) != 0);
              break;
            }
          std::vector<int32_t> bad = acts;  // stage out of range -> malformed
          bad[0] = S;
          CHECK(ddl_sched_verify(bad.data(), need, S) == -1000000);
        }
      }
  CHECK(ddl_sched_build(2, 0, 4, nullptr, 0) == 0);
}

static void epochs() {
  for (int G : {1, 3, 8})
    for (int count : {1, 7, 100, 6250})
      for (int batch : {1, 32, 100, 128}) {
        std::vector<int32_t> idx((size_t)G * count);
        for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int32_t)i;
        std::vector<uint64_t> seeds(G);
        for (int g = 0; g < G; ++g) seeds[g] = 1234 + g;
        const int steps = (count + batch - 1) / batch;
        std::vector<int32_t> out((size_t)steps * G * batch);
        CHECK(ddl_plan_epoch(idx.data(), G, count, batch, seeds.data(), 1, out.data()) == steps);
        for (int g = 0; g < G; ++g) {  // each client's plan is a permutation of its own ids
          std::vector<char> seen(count, 0);
          int pads = 0;
          for (int st = 0; st < steps; ++st)
            for (int b = 0; b < batch; ++b) {
              const int32_t v = out[((size_t)st * G + g) * batch + b];
              if (v < 0) { ++pads; continue; }
              const int32_t k = v - g * count;
              CHECK(k >= 0 && k < count);
              if (k >= 0 && k < count) { CHECK(!seen[k]); seen[k] = 1; }
            }
          CHECK(pads == steps * batch - count);
        }
      }
}

static void buckets() {
  std::vector<int64_t> sizes;
  for (int i = 0; i < 200; ++i) sizes.push_back(1 + (i * 7919) % 100000);
  for (int64_t cap : {1LL, 4096LL, 1LL << 20, 25LL << 20, 1LL << 40}) {
    std::vector<int32_t> out(sizes.size());
    const int nb = ddl_bucket_plan(sizes.data(), (int)sizes.size(), cap, 4, out.data());
    CHECK(nb >= 1 && out.back() == nb - 1);
    for (size_t i = 1; i < out.size(); ++i) CHECK(out[i] == out[i - 1] || out[i] == out[i - 1] + 1);
  }
  CHECK(ddl_bucket_plan(nullptr, 0, 1024, 4, nullptr) == 0);
}

static void markov() {
  const int V = 40, br = 5, B = 3, S = 64;
  std::vector<int64_t> next((size_t)V * br);
  std::vector<double> cum((size_t)V * br);
  for (int v = 0; v < V; ++v)
    for (int k = 0; k < br; ++k) {
      next[(size_t)v * br + k] = (v * 31 + k * 7) % V;
      cum[(size_t)v * br + k] = (k + 1.0) / br;
    }
  std::vector<int64_t> cur0 = {0, 5, V - 1};
  std::vector<double> U((size_t)B * S);
  for (size_t i = 0; i < U.size(); ++i) U[i] = (double)((i * 2654435761u) % 1000) / 1000.0;
  U[7] = 1.0;  // past the last cumulative bucket: must clamp to br-1, not read past the row
  std::vector<int64_t> out((size_t)B * S);
  CHECK(ddl_markov_walk(next.data(), cum.data(), br, cur0.data(), U.data(), B, S, 1, out.data()) == 0);
  for (int b = 0; b < B; ++b) {
    CHECK(out[(size_t)b * S] == 1);
    for (int t = 1; t < S; ++t) CHECK(out[(size_t)b * S + t] >= 0 && out[(size_t)b * S + t] < V);
  }
}

int main() {
  CHECK(ddl_runtime_version() >= 1);
  schedules();
  epochs();
  buckets();
  markov();
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("runtime sanitize ok\n");
  return 0;
}
