// Host-runtime self test, built with -fsanitize=address,undefined (and, separately,
// -fsanitize=thread) by tests/test_host_sanitize.py (the GPU pool has
// no GPU ASan / xnack+, so sanitizers cover the host C++ code).
//
// It includes the library source directly so the sanitizers instrument every line
// of it, then checks
//   * the rolling mean / std / median against an O(n*w) recomputation, with NaN
//     gaps, min_periods, windows longer than the series and the periodic re-sum,
//     single- and multi-threaded (the threaded path is what TSan watches);
//   * CRC32C: the standard check value, hardware vs slicing-by-8 on every length
//     and misalignment 0..7, and the TFRecord masking;
//   * concurrent first use of the CRC tables from several threads.
#include "../host/gnnqc_host.cpp"

#include <cstdio>
#include <cstdlib>
#include <random>

static int g_fail = 0;
#define CHECK(c, ...)                                           \
  do {                                                          \
    if (!(c)) {                                                 \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                        \
      std::fprintf(stderr, "\n");                               \
      if (++g_fail > 20) std::exit(1);                          \
    }                                                           \
  } while (0)

static bool close_or_nan(float a, double b, double tol) {
  if (std::isnan(a) || std::isnan(b)) return std::isnan(a) && std::isnan(b);
  return std::fabs(a - b) <= tol * (1.0 + std::fabs(b));
}

static void naive(const float* x, int64_t w, int64_t minp, int64_t t, double* mean, double* sd, double* med) {
  std::vector<double> v;
  for (int64_t k = std::max<int64_t>(0, t - w + 1); k <= t; ++k)
    if (!std::isnan(x[k])) v.push_back(x[k]);
  const double qnan = std::nan("");
  if (v.empty() || static_cast<int64_t>(v.size()) < minp) {
    *mean = *sd = *med = qnan;
    return;
  }
  double s = 0, s2 = 0;
  for (double a : v) { s += a; s2 += a * a; }
  const double m = s / v.size();
  *mean = m;
  *sd = std::sqrt(std::max(s2 / v.size() - m * m, 0.0));
  std::sort(v.begin(), v.end());
  const size_t c = v.size();
  *med = (c & 1) ? v[c / 2] : 0.5 * (v[c / 2 - 1] + v[c / 2]);
}

static void test_rolling(int64_t rows, int64_t n, int64_t w, int64_t minp, int threads, unsigned seed) {
  std::mt19937 rng(seed);
  std::normal_distribution<float> nd(10.f, 3.f);
  std::uniform_real_distribution<float> u(0.f, 1.f);
  std::vector<float> x(rows * n);
  for (auto& a : x) a = u(rng) < 0.1f ? std::nanf("") : nd(rng);
  // a long NaN gap in row 0 (the window empties completely)
  for (int64_t t = n / 3; t < std::min(n, n / 3 + w + 5); ++t) x[t] = std::nanf("");
  std::vector<float> mean(rows * n), sd(rows * n), med(rows * n);
  gq_rolling_stats(x.data(), rows, n, w, minp, mean.data(), sd.data(), med.data(), threads);
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t t = 0; t < n; ++t) {
      double m, s, md;
      naive(&x[r * n], w, minp, t, &m, &s, &md);
      const int64_t i = r * n + t;
      CHECK(close_or_nan(mean[i], m, 1e-5), "mean r=%ld t=%ld got %g want %g", (long)r, (long)t, mean[i], m);
      CHECK(close_or_nan(sd[i], s, 1e-3), "std r=%ld t=%ld got %g want %g", (long)r, (long)t, sd[i], s);
      CHECK(close_or_nan(med[i], md, 1e-6), "median r=%ld t=%ld got %g want %g", (long)r, (long)t, med[i], md);
    }
  // null outputs are allowed (median only)
  std::vector<float> med2(rows * n);
  gq_rolling_stats(x.data(), rows, n, w, minp, nullptr, nullptr, med2.data(), threads);
  CHECK(std::memcmp(med.data(), med2.data(), med.size() * sizeof(float)) == 0, "median-only run differs");
}

static void test_crc() {
  const uint8_t* check = reinterpret_cast<const uint8_t*>("123456789");
  CHECK(gq_crc32c(check, 9, 0) == 0xE3069283u, "crc32c check value");
  CHECK(gq_crc32c_sw(check, 9, 0) == 0xE3069283u, "sw crc32c check value");
  std::vector<uint8_t> buf(4096 + 8);
  std::mt19937 rng(7);
  for (auto& b : buf) b = static_cast<uint8_t>(rng());
  for (int off = 0; off < 8; ++off)
    for (uint64_t n = 0; n < 300; ++n) {
      const uint8_t* p = buf.data() + off;
      CHECK(gq_crc32c(p, n, 0) == gq_crc32c_sw(p, n, 0), "hw/sw crc differ off=%d n=%lu", off, (unsigned long)n);
      const uint64_t h = n / 2;  // incremental == one-shot
      CHECK(gq_crc32c(p + h, n - h, gq_crc32c(p, h, 0)) == gq_crc32c(p, n, 0), "incremental crc n=%lu",
            (unsigned long)n);
    }
  const uint32_t c = gq_crc32c(buf.data(), 4096, 0);
  CHECK(gq_masked_crc32c(buf.data(), 4096) == ((c >> 15) | (c << 17)) + 0xa282ead8u, "masked crc");
}

static void test_crc_threads() {
  std::vector<uint8_t> buf(1000);
  for (size_t i = 0; i < buf.size(); ++i) buf[i] = static_cast<uint8_t>(i * 31 + 7);
  std::vector<uint32_t> got(8);
  std::vector<std::thread> th;
  for (int i = 0; i < 8; ++i) th.emplace_back([&, i] { got[i] = gq_crc32c_sw(buf.data(), buf.size(), 0); });
  for (auto& t : th) t.join();
  const uint32_t want = gq_crc32c(buf.data(), buf.size(), 0);
  for (int i = 0; i < 8; ++i) CHECK(got[i] == want, "threaded sw crc %d", i);
}

int main() {
  test_crc_threads();  // first use of the tables happens concurrently here
  test_crc();
  test_rolling(3, 500, 37, 1, 1, 1);
  test_rolling(7, 700, 60, 5, 4, 2);
  test_rolling(2, 120, 500, 1, 2, 3);  // window longer than the series
  test_rolling(1, 8300, 64, 1, 1, 4);  // crosses the periodic exact re-sum at t=8191
  test_rolling(5, 50, 1, 1, 3, 5);     // window of one
  if (g_fail) {
    std::fprintf(stderr, "%d failures\n", g_fail);
    return 1;
  }
  std::printf("host sanitize self-test OK\n");
  return 0;
}
