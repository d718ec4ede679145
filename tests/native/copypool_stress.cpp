// Stress test of klf::CopyPool (the staging copy workers) for the host sanitizers:
// many caller threads, random piece sizes, every byte checked.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "../../klogs_amd/csrc/klf_copypool.hpp"

int main() {
  klf::CopyPool pool(3);
  std::vector<std::thread> th;
  int bad = 0;
  std::mutex mu;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      std::mt19937 rng(t);
      std::vector<uint8_t> src(8 << 20), dst(8 << 20);
      for (auto& b : src) b = (uint8_t)rng();
      for (int it = 0; it < 200; ++it) {
        const size_t n = rng() % src.size();
        std::fill(dst.begin(), dst.begin() + n, 0);
        pool.copy(dst.data(), src.data(), n);
        if (memcmp(dst.data(), src.data(), n)) { std::lock_guard<std::mutex> g(mu); ++bad; }
      }
    });
  for (auto& x : th) x.join();
  printf("copypool: %s\n", bad ? "FAIL" : "ok");
  return bad ? 1 : 0;
}
