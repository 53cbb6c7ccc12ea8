// Host request-path microbenchmark: ns per row of the risk.v1 ScoreBatch parse (wire.cpp), the
// identifier digests alone, and the ScoreBatchResponse serializer, on 8192-row batches shaped
// like tools/bench_e2e.py's payloads (UUID account ids, device / fingerprint / ip strings).
// Build: g++ -std=c++17 -O2 -Icsrc/include tools/probe/wire_bench.cpp csrc/runtime/wire.cpp -o /tmp/wire_bench
#include <chrono>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

#include "../../csrc/runtime/pb.h"
#include "../../csrc/runtime/wire.h"
#include "../../csrc/runtime/xxh64.h"

using namespace igp;

static double now_ns() {
  return std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int B = 8192, reps = argc > 1 ? atoi(argv[1]) : 100;
  std::mt19937_64 rng(1);
  pb::Writer batch;
  const char* types[4] = {"deposit", "withdraw", "bet", "win"};
  for (int i = 0; i < B; ++i) {
    const uint64_t a = rng() % 1000000, d = rng() % 6;
    char uuid[40];
    snprintf(uuid, sizeof uuid, "%08llx-%04llx-4%03llx-8%03llx-%012llx", (unsigned long long)(rng() & 0xffffffff),
             (unsigned long long)(rng() & 0xffff), (unsigned long long)(rng() & 0xfff),
             (unsigned long long)(rng() & 0xfff), (unsigned long long)(rng() & 0xffffffffffffULL));
    pb::Writer tx;
    tx.str(1, uuid);
    tx.i64(3, int64_t(100 + rng() % 500000));
    tx.str(4, types[rng() % 4]);
    tx.str(5, "EUR");
    tx.str(8, "10." + std::to_string(a % 250) + "." + std::to_string(a / 250 % 250) + "." + std::to_string(d));
    tx.str(9, "dev-" + std::to_string(a) + "-" + std::to_string(d));
    tx.str(10, "fp-" + std::to_string(a) + "-" + std::to_string(d));
    tx.str(12, "s-" + std::to_string(a));
    batch.msg(1, tx.buf);
  }
  const std::string& bytes = batch.buf;
  std::vector<wire::TxRow> rows;
  rows.reserve(B);
  double best = 1e30;
  for (int r = 0; r < reps; ++r) {
    rows.clear();
    const double t = now_ns();
    wire::parse_batch_rows(bytes.data(), bytes.size(), rows);
    best = std::min(best, now_ns() - t);
  }
  printf("parse_batch_rows      %6.1f ns/row (%zu B/row)\n", best / B, bytes.size() / B);
  // digests alone
  double hb = 1e30;
  uint64_t sink = 0;
  for (int r = 0; r < reps; ++r) {
    const double t = now_ns();
    for (const auto& x : rows) sink += id_hash(x.account, SEED_ACCOUNT) ^ sink;
    hb = std::min(hb, now_ns() - t);
  }
  printf("  account digest      %6.1f ns/row\n", hb / B);
  std::vector<ResultRec> res(B);
  std::vector<FeatRec> feat(B);
  for (int i = 0; i < B; ++i) {
    res[i].packed = uint32_t(rng() & 0xff) | (uint32_t(rng() & 0xff) << 8) | (uint32_t(rng() & 3) << 16) |
                    (uint32_t(rng() & 0x7) << 20);
    res[i].ml = float(rng() % 1000) / 1000.f;
    FeatRec& f = feat[i];
    std::memset(&f, 0, sizeof f);
    f.tx_count_1m = rng() % 5; f.tx_count_5m = rng() % 10; f.tx_count_1h = rng() % 40;
    f.tx_sum_1h = rng() % 1000000; f.tx_avg_1h = float(rng() % 10000); f.unique_devices_24h = 1 + rng() % 3;
    f.unique_ips_24h = 1 + rng() % 3; f.account_age_days = rng() % 900; f.device_age_days = rng() % 300;
    f.total_deposits = rng() % 10000000; f.total_withdrawals = rng() % 1000000;
    f.net_deposit = f.total_deposits - f.total_withdrawals; f.deposit_count = rng() % 100;
    f.withdraw_count = rng() % 20; f.time_since_last_tx = rng() % 3600; f.avg_bet_size = float(rng() % 5000);
    f.win_rate = 0.47f;
  }
  double sb = 1e30;
  size_t len = 0;
  for (int r = 0; r < reps; ++r) {
    const double t = now_ns();
    len = wire::batch_response_scratch(res.data(), feat.data(), nullptr, 3, B).size();
    sb = std::min(sb, now_ns() - t);
  }
  printf("batch response        %6.1f ns/row (%zu B/row)\n", sb / B, len / B);
  printf("(sink %llu)\n", (unsigned long long)(sink & 1));
  return 0;
}
