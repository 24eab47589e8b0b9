// sanitize_main.cpp — ASan + UBSan driver (TEST INFRASTRUCTURE ONLY; SURVEY §5 "Race detection /
// sanitizers": test the C++ under ASan/UBSan, Java's signed-overflow semantics emulated explicitly).
// Built by `make -C oracle sanitize` with -fsanitize=address,undefined and run by tests/test_sanitizers.py.
// It drives the oracle through every operator shape (tumbling / sliding / sessions, lateness, purging,
// side output, first-element, minBy/maxBy, HyperLogLog, t-digest, count windows, the multi-threaded
// baseline) on a seeded stream with extreme keys and timestamps, and checks the host-side arithmetic the
// library shares with the device code (make_div_inv, flink_amd/csrc/fw_internal.h) against 128-bit division.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../flink_amd/csrc/fw_internal.h"
#include "window_oracle.h"

static uint64_t sm(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static int check_div_inv() {
  // the quotient the device computes from (m, l): t1 = mulhi(m, n); (t1 + ((n - t1) >> 1)) >> (l - 1)
  int bad = 0;
  const uint64_t ds[] = {1, 2, 3, 7, 1000, 60000, 1000003, 86400000ull, (1ull << 40) + 5, ~0ull >> 1};
  for (uint64_t d : ds) {
    uint64_t m;
    int32_t l;
    make_div_inv(d, &m, &l);
    for (int i = 0; i < 20000; i++) {
      const uint64_t n = i < 10 ? (uint64_t)i : (i < 20 ? ~0ull - (uint64_t)(i - 10) : sm((uint64_t)i * 7919u + d));
      uint64_t q;
      if (l == 0) {
        q = n;
      } else {
        const uint64_t t1 = (uint64_t)(((unsigned __int128)m * n) >> 64);
        q = (t1 + ((n - t1) >> 1)) >> (l - 1);
      }
      if (q != n / d) bad++;
    }
  }
  return bad;
}

static void run(oracle_cfg cfg, int n, uint64_t seed) {
  void* op = oracle_create(&cfg);
  std::vector<int64_t> k(n), t(n), v(n);
  int64_t mx = INT64_MIN + 5000;
  for (int b = 0; b < 4; b++) {
    for (int i = 0; i < n; i++) {
      const uint64_t r = sm(seed ^ ((uint64_t)(b * n + i) << 2));
      k[i] = (int64_t)(r % 97) - 48;
      if (i % 31 == 0) k[i] = (i & 1) ? INT64_MAX : INT64_MIN;  // extreme keys
      t[i] = 1000000 + (int64_t)((b * n + i) / 4) - (int64_t)(sm(r) % 300);
      if (b == 3 && i % 53 == 0) t[i] = INT64_MAX - 1750 + (int64_t)(r % 100);  // cleanup-time overflow
      const int64_t x = (int64_t)sm(r + 1);
      if (cfg.value_type == OR_VAL_F64) {
        const double d = (double)(x % 1000000) / 7.0;
        memcpy(&v[i], &d, 8);
      } else {
        v[i] = cfg.value_type == OR_VAL_I32 ? (int64_t)(int32_t)x : x;
      }
      if (t[i] > mx) mx = t[i];
    }
    oracle_process(op, k.data(), t.data(), v.data(), n);
    oracle_watermark(op, mx - 200);
  }
  oracle_watermark(op, INT64_MAX);
  std::vector<oracle_row> rows((size_t)oracle_num_rows(op));
  if (!rows.empty()) oracle_get_rows(op, rows.data());
  if (cfg.aggregate == OR_AGG_TDIGEST && !rows.empty()) {
    std::vector<double> s(64);
    std::vector<int64_t> w(64);
    oracle_row_digest(op, 0, s.data(), w.data(), 64);
  }
  std::vector<oracle_side_row> side((size_t)oracle_num_side_rows(op));
  if (!side.empty()) oracle_get_side_rows(op, side.data());
  oracle_destroy(op);
}

int main() {
  const int bad = check_div_inv();
  if (bad) {
    fprintf(stderr, "make_div_inv: %d wrong quotients\n", bad);
    return 1;
  }
  oracle_cfg base{};
  base.td_delta = 100;
  base.td_q[0] = 0.5;
  base.td_q[1] = 0.9;
  base.td_q[2] = 0.99;
  auto cfg = [&](int a, int vt, int64_t size, int64_t slide, int64_t gap, int64_t late, int purge, int side, int agg) {
    oracle_cfg c = base;
    c.assigner = a;
    c.value_type = vt;
    c.size = size;
    c.slide = slide;
    c.gap = gap;
    c.lateness = late;
    c.purging = purge;
    c.side_output = side;
    c.aggregate = agg;
    c.hll_p = 10;
    return c;
  };
  run(cfg(OR_TUMBLING, OR_VAL_I64, 1000, 1000, 0, 0, 0, 0, OR_AGG_COUNT_SUM_MIN_MAX), 3000, 1);
  run(cfg(OR_TUMBLING, OR_VAL_I32, 1000, 1000, 0, 700, 1, 1, OR_AGG_FIRST), 3000, 2);
  run(cfg(OR_SLIDING, OR_VAL_F64, 3000, 1000, 0, 0, 0, 0, OR_AGG_COUNT_SUM_MIN_MAX), 2000, 3);
  run(cfg(OR_SLIDING, OR_VAL_I64, 2000, 500, 0, 300, 0, 1, OR_AGG_MINBY), 2000, 4);
  run(cfg(OR_SESSION, OR_VAL_F64, 0, 0, 300, 200, 1, 1, OR_AGG_MAXBY), 3000, 5);
  run(cfg(OR_SESSION, OR_VAL_I64, 0, 0, 50, 0, 0, 0, OR_AGG_FIRST_MAX), 3000, 6);
  run(cfg(OR_TUMBLING, OR_VAL_I64, 1000, 1000, 0, 0, 0, 0, OR_AGG_HLL), 3000, 7);
  run(cfg(OR_TUMBLING, OR_VAL_F64, 1000, 1000, 0, 0, 0, 0, OR_AGG_TDIGEST), 6000, 8);
  {  // count windows (a14)
    void* cw = oracle_count_create(10, 5, 1, OR_VAL_I32);
    std::vector<int64_t> k(5000), v(5000);
    for (int i = 0; i < 5000; i++) {
      k[i] = (int64_t)(sm(i) % 170);
      v[i] = 1;
    }
    oracle_count_process(cw, k.data(), v.data(), 5000);
    std::vector<oracle_row> rows((size_t)oracle_count_num_rows(cw));
    if (!rows.empty()) oracle_count_get_rows(cw, rows.data());
    oracle_count_destroy(cw);
  }
  {  // the multi-threaded CPU baseline (p = 4 subtasks)
    oracle_cfg c = cfg(OR_TUMBLING, OR_VAL_I64, 1000, 1000, 0, 0, 0, 0, OR_AGG_COUNT_SUM_MIN_MAX);
    const int n = 40000;
    std::vector<int64_t> k(n), t(n), v(n), wms(4);
    for (int i = 0; i < n; i++) {
      k[i] = (int64_t)(sm(i) % 1000);
      t[i] = i / 10;
      v[i] = (int64_t)sm(i + 1);
    }
    for (int b = 0; b < 4; b++) wms[b] = (int64_t)((b + 1) * n / 4) / 10 - 200;
    int64_t late = 0;
    oracle_run_parallel(&c, k.data(), t.data(), v.data(), n, n / 4, wms.data(), 4, 128, 4, &late);
  }
  printf("sanitized run ok\n");
  return 0;
}
