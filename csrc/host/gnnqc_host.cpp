// gnnqc host runtime library (C ABI, loaded with ctypes).
//
// Native replacements for the CPU-side pieces the reference delegates to C
// libraries:
//   * trailing rolling mean / std / median with min_periods and NaN skipping
//     (xarray+bottleneck in libs/preprocessing_functions.py:135-140,162-172),
//     multithreaded over sensors; the median keeps a sorted window (binary search
//     + memmove), O(w) per step with a tiny constant.
//   * CRC32C (Castagnoli) with the TFRecord / LevelDB masking used by TF's record
//     files and TensorBundle/SSTable checkpoints (model_*/variables/variables.index).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#if defined(__x86_64__) && defined(__SSE4_2__)
#include <nmmintrin.h>
#define GQ_HW_CRC 1
#endif

namespace {

void rolling_row(const float* x, int64_t n, int64_t w, int64_t minp, float* mean, float* sd,
                 float* med) {
  std::vector<float> win;
  win.reserve(static_cast<size_t>(std::min<int64_t>(w, n)) + 1);
  double s = 0.0, s2 = 0.0;
  int64_t cnt = 0;
  const float qnan = std::nanf("");
  for (int64_t t = 0; t < n; ++t) {
    const float v = x[t];
    if (!std::isnan(v)) {
      s += v;
      s2 += static_cast<double>(v) * v;
      ++cnt;
      if (med) win.insert(std::upper_bound(win.begin(), win.end(), v), v);
    }
    const int64_t old = t - w;
    if (old >= 0) {
      const float u = x[old];
      if (!std::isnan(u)) {
        s -= u;
        s2 -= static_cast<double>(u) * u;
        --cnt;
        if (med) win.erase(std::lower_bound(win.begin(), win.end(), u));
      }
    }
    // periodic exact resum to bound floating drift of the running sums
    if ((t & 8191) == 8191 && (mean || sd)) {
      s = 0.0; s2 = 0.0;
      for (int64_t k = std::max<int64_t>(0, t - w + 1); k <= t; ++k) {
        if (!std::isnan(x[k])) { s += x[k]; s2 += static_cast<double>(x[k]) * x[k]; }
      }
    }
    const bool ok = cnt >= minp && cnt > 0;
    if (mean) mean[t] = ok ? static_cast<float>(s / cnt) : qnan;
    if (sd) {
      if (ok) {
        double m = s / cnt;
        double var = s2 / cnt - m * m;
        sd[t] = static_cast<float>(std::sqrt(std::max(var, 0.0)));
      } else {
        sd[t] = qnan;
      }
    }
    if (med) {
      const size_t c = win.size();
      if (ok && c > 0) {
        med[t] = (c & 1) ? win[c / 2] : 0.5f * (win[c / 2 - 1] + win[c / 2]);
      } else {
        med[t] = qnan;
      }
    }
  }
}

struct CrcTable {
  uint32_t v[8][256];
  CrcTable();
};

CrcTable::CrcTable() {
  uint32_t (&crc_table)[8][256] = v;
  const uint32_t poly = 0x82F63B78u;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : (c >> 1);
    crc_table[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t)
      crc_table[t][i] = (crc_table[t - 1][i] >> 8) ^ crc_table[0][crc_table[t - 1][i] & 0xFF];
}

// slicing-by-8 tables, built once (thread-safe function-local static: the record
// readers may call in from several Python threads)
const uint32_t (&crc_tables())[8][256] {
  static const CrcTable tab;
  return tab.v;
}

uint32_t crc32c_sw(uint32_t crc, const uint8_t* p, size_t n) {
  const uint32_t (&crc_table)[8][256] = crc_tables();
  crc = ~crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= crc;
    crc = crc_table[7][v & 0xFF] ^ crc_table[6][(v >> 8) & 0xFF] ^ crc_table[5][(v >> 16) & 0xFF] ^
          crc_table[4][(v >> 24) & 0xFF] ^ crc_table[3][(v >> 32) & 0xFF] ^
          crc_table[2][(v >> 40) & 0xFF] ^ crc_table[1][(v >> 48) & 0xFF] ^ crc_table[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) crc = (crc >> 8) ^ crc_table[0][(crc ^ *p++) & 0xFF];
  return ~crc;
}

}  // namespace

extern "C" {

int gq_version() { return 1; }

// portable slicing-by-8 path (used where SSE4.2 is absent; tested against the hardware path)
uint32_t gq_crc32c_sw(const uint8_t* data, uint64_t n, uint32_t init) { return crc32c_sw(init, data, n); }

// x: [rows, n] row-major. Any output pointer may be null.
void gq_rolling_stats(const float* x, int64_t rows, int64_t n, int64_t window, int64_t min_periods,
                      float* mean, float* sd, float* med, int32_t nthreads) {
  if (nthreads <= 0) nthreads = static_cast<int32_t>(std::max(1u, std::thread::hardware_concurrency()));
  nthreads = static_cast<int32_t>(std::min<int64_t>(nthreads, std::max<int64_t>(rows, 1)));
  auto work = [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      rolling_row(x + r * n, n, window, min_periods, mean ? mean + r * n : nullptr,
                  sd ? sd + r * n : nullptr, med ? med + r * n : nullptr);
    }
  };
  if (nthreads == 1) {
    work(0, rows);
    return;
  }
  std::vector<std::thread> pool;
  // rows are independent: hand them out round-robin in contiguous chunks
  const int64_t chunk = (rows + nthreads - 1) / nthreads;
  for (int32_t i = 0; i < nthreads; ++i) {
    const int64_t r0 = i * chunk, r1 = std::min(rows, r0 + chunk);
    if (r0 >= r1) break;
    pool.emplace_back(work, r0, r1);
  }
  for (auto& th : pool) th.join();
}

uint32_t gq_crc32c(const uint8_t* data, uint64_t n, uint32_t init) {
#ifdef GQ_HW_CRC
  uint64_t crc = ~init;
  const uint8_t* p = data;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    crc = _mm_crc32_u64(crc, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = static_cast<uint32_t>(crc);
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
#else
  return crc32c_sw(init, data, n);
#endif
}

// TFRecord / LevelDB masked crc
uint32_t gq_masked_crc32c(const uint8_t* data, uint64_t n) {
  const uint32_t c = gq_crc32c(data, n, 0);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

}  // extern "C"
