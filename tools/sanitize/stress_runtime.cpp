// Host-side race / memory-safety stress for the native runtime (the reference runs
// `go test -race`, Makefile:34-36; this is the C++ equivalent under TSan and ASan+UBSan).
//
// Built and run by `make sanitize` (tools/sanitize/run.sh) with clang++ -fsanitize=thread and
// -fsanitize=address,undefined over the same host sources the extension links
// (csrc/cpu/*.cpp, csrc/runtime/miner_common.cpp). No GPU code: the HIP miner's host loop shares
// MinerBase / ShareQueue / JobTemplate with the CPU miner, which is what is exercised here.
//
// Properties checked (exit status != 0 on any violation, so the sanitizer run is also the test):
//  1. ShareQueue under 4 producers / 2 consumers: pushed == drained + dropped, nothing invented.
//  2. Job-epoch protocol: while the control thread switches jobs every ~1 ms (new work, re-issued
//     work with a new target/epoch = SV2 SetTarget, pause = nullptr), every share the miner emits
//     names an epoch that was issued, carries that epoch's job id, and its header rebuilt from THAT
//     epoch's template hashes to the reported hash and meets THAT epoch's target.
//  3. No duplicates: a (work, extranonce2, version, ntime, nonce) tuple is never emitted twice, even
//     across re-issues of the same work and pause/resume (the cursor must not restart).
//  4. AEAD round trip + tamper rejection and scrypt/HMAC/PBKDF2 on odd lengths (ASan coverage).
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "otedama/aead.h"
#include "otedama/runtime.h"
#include "otedama/sha256.h"

using namespace otedama;

static int g_fail = 0;
#define CHECK(c, ...)                                   \
  do {                                                  \
    if (!(c)) {                                         \
      if (g_fail < 20) {                                \
        std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
        std::fprintf(stderr, __VA_ARGS__);              \
        std::fprintf(stderr, "\n");                     \
      }                                                 \
      ++g_fail;                                         \
    }                                                   \
  } while (0)

static ShareRecord fake_share(uint64_t i) {
  ShareRecord s{};
  s.epoch = i;
  s.job_id = "j" + std::to_string(i);
  s.nonce = uint32_t(i);
  s.device_id = "q";
  return s;
}

static void test_share_queue() {
  ShareQueue q(1000);
  constexpr int kProd = 4, kPer = 20000;
  std::atomic<int> pushed{0}, live_producers{kProd};
  std::atomic<uint64_t> drained{0};
  std::vector<std::thread> ths;
  for (int p = 0; p < kProd; ++p)
    ths.emplace_back([&, p] {
      for (int i = 0; i < kPer; ++i)
        if (q.push(fake_share(uint64_t(p) * kPer + i))) pushed.fetch_add(1);
      live_producers.fetch_sub(1);
    });
  for (int c = 0; c < 2; ++c)
    ths.emplace_back([&] {
      while (live_producers.load() > 0 || q.size() > 0) {
        auto v = q.drain(64);
        for (auto& s : v) CHECK(s.job_id == "j" + std::to_string(s.epoch), "share queue corrupted a record");
        drained.fetch_add(v.size());
      }
    });
  for (auto& t : ths) t.join();
  CHECK(uint64_t(pushed.load()) == drained.load(), "pushed %d drained %llu", pushed.load(),
        (unsigned long long)drained.load());
  CHECK(uint64_t(pushed.load()) + q.dropped() == uint64_t(kProd) * kPer, "pushed+dropped != offered");
}

struct Issued {
  std::shared_ptr<const JobTemplate> job;
  int work;  // distinct search space id (re-issues of the same work share it)
};

static std::shared_ptr<JobTemplate> make_work(std::mt19937_64& rng, int work, uint64_t epoch, uint8_t top) {
  auto j = std::make_shared<JobTemplate>();
  j->epoch = epoch;
  j->job_id = "w" + std::to_string(work) + "e" + std::to_string(epoch);
  j->algo = Algo::kSha256d;
  for (auto& b : j->header) b = uint8_t(rng());
  std::memset(j->target, 0xff, 32);
  j->target[31] = top;  // top=0 -> 1/256 of hashes are shares
  j->has_coinbase = true;
  j->coinb1.assign(41, uint8_t(work));
  j->coinb2.assign(23, uint8_t(work * 7));
  j->extranonce1 = {1, 2, 3, 4};
  j->extranonce2_size = 2;
  j->merkle_branches.assign(2, std::vector<uint8_t>(32, uint8_t(work + 1)));
  j->version_mask = (work % 2) ? 0x1fffe000u : 0;
  j->ntime_roll = (work % 3) ? 7 : 0;
  return j;
}

static void rebuild_header(const JobTemplate& j, const ShareRecord& s, uint8_t out[80]) {
  std::memcpy(out, j.header, 80);
  uint8_t root[32];
  merkle_root_from_coinbase(j, s.extranonce2, root);
  std::memcpy(out + 36, root, 32);
  store_le32(out, s.version);
  store_le32(out + 68, s.ntime);
  store_le32(out + 76, s.nonce);
}

static void test_job_epochs(int threads, double seconds) {
  CpuMiner m(threads, "cpu-stress", 1 << 15);
  std::mutex mu;
  std::map<uint64_t, Issued> issued;
  std::mt19937_64 rng(1234);
  uint64_t epoch = 0;
  int work = 0;
  std::shared_ptr<JobTemplate> cur = make_work(rng, work, ++epoch, 0);
  issued[cur->epoch] = {cur, work};
  m.set_job(cur);
  m.start();

  std::set<std::tuple<int, uint64_t, uint32_t, uint32_t, uint32_t>> seen;
  uint64_t shares = 0, stale = 0, switches = 0;
  auto check_batch = [&](const std::vector<ShareRecord>& v, uint64_t current_epoch) {
    std::lock_guard<std::mutex> g(mu);
    for (const auto& s : v) {
      ++shares;
      auto it = issued.find(s.epoch);
      CHECK(it != issued.end(), "share names unissued epoch %llu", (unsigned long long)s.epoch);
      if (it == issued.end()) continue;
      const JobTemplate& j = *it->second.job;
      if (s.epoch != current_epoch) ++stale;
      CHECK(s.job_id == j.job_id, "epoch %llu: job id %s != %s", (unsigned long long)s.epoch, s.job_id.c_str(),
            j.job_id.c_str());
      CHECK(s.device_id == "cpu-stress", "device id");
      uint8_t hdr[80], h[32];
      rebuild_header(j, s, hdr);
      sha256d(hdr, 80, h);
      CHECK(std::memcmp(h, s.hash, 32) == 0, "epoch %llu nonce %08x: reported hash is not the header's",
            (unsigned long long)s.epoch, s.nonce);
      CHECK(le256_leq(h, j.target), "epoch %llu nonce %08x: share misses its epoch's target",
            (unsigned long long)s.epoch, s.nonce);
      CHECK((s.version & ~j.version_mask) == (load_le32(j.header) & ~j.version_mask), "version outside mask");
      const uint32_t nt0 = load_le32(j.header + 68);
      CHECK(s.ntime >= nt0 && s.ntime <= nt0 + j.ntime_roll, "ntime outside roll window");
      auto key = std::make_tuple(it->second.work, s.extranonce2, s.version, s.ntime, s.nonce);
      CHECK(seen.insert(key).second, "duplicate share: work %d en2 %llu nonce %08x (epoch %llu)", it->second.work,
            (unsigned long long)s.extranonce2, s.nonce, (unsigned long long)s.epoch);
    }
  };

  const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(seconds);
  std::uniform_int_distribution<int> op(0, 9);
  bool paused = false;
  while (std::chrono::steady_clock::now() < t_end) {
    std::this_thread::sleep_for(std::chrono::microseconds(300 + rng() % 1500));
    const int o = op(rng);
    std::shared_ptr<JobTemplate> next;
    if (o < 5) {  // new work (clean_jobs)
      next = make_work(rng, ++work, ++epoch, 0);
    } else if (o < 8) {  // same work, new target / epoch (SV2 SetTarget / V1 set_difficulty)
      next = std::make_shared<JobTemplate>(*cur);
      next->epoch = ++epoch;
      next->job_id = "w" + std::to_string(work) + "e" + std::to_string(epoch);
      next->target[31] = uint8_t(rng() % 2);
    } else if (o == 8 && !paused) {  // pause (curtailment / arbitration)
      m.set_job(nullptr);
      paused = true;
      continue;
    } else {  // resume the current job unchanged
      next = cur;
    }
    check_batch(m.poll(1 << 15), cur->epoch);  // before the switch: `stale` counts real races
    {
      std::lock_guard<std::mutex> g(mu);
      issued[next->epoch] = {next, work};
    }
    cur = next;
    paused = false;
    m.set_job(cur);
    ++switches;
  }
  m.stop();
  check_batch(m.poll(1 << 16), cur->epoch);
  const MinerStats st = m.stats();
  CHECK(!st.faulted, "miner faulted: %s", st.error.c_str());
  CHECK(shares > 100, "too few shares to mean anything (%llu)", (unsigned long long)shares);
  CHECK(st.shares == shares + st.dropped, "stats.shares %llu != polled %llu + dropped %llu",
        (unsigned long long)st.shares, (unsigned long long)shares, (unsigned long long)st.dropped);
  std::printf("job-epoch stress: %llu switches, %llu shares (%llu polled after their epoch was superseded, all self-consistent), "
              "%llu hashes, %d distinct works\n",
              (unsigned long long)switches, (unsigned long long)shares, (unsigned long long)stale,
              (unsigned long long)st.hashes, work + 1);
}

static void test_crypto_memory() {
  std::mt19937_64 rng(7);
  for (int kind = 0; kind < 2; ++kind)
    for (size_t len : {0ul, 1ul, 15ul, 16ul, 17ul, 63ul, 64ul, 65ul, 1000ul}) {
      std::string key(32, '\0'), nonce(12, '\0'), plain(len, '\0'), aad(len % 7, 'a');
      for (auto& c : key) c = char(rng());
      for (auto& c : nonce) c = char(rng());
      for (auto& c : plain) c = char(rng());
      const std::string sealed = aead_seal(AeadKind(kind), key, nonce, plain, aad);
      CHECK(sealed.size() == len + kAeadTagBytes, "sealed size");
      std::string back;
      CHECK(aead_open(AeadKind(kind), key, nonce, sealed, aad, &back) && back == plain, "aead round trip");
      std::string bad = sealed;
      bad[rng() % bad.size()] ^= 1;
      CHECK(!aead_open(AeadKind(kind), key, nonce, bad, aad, &back), "tampered ciphertext accepted");
      CHECK(!aead_open(AeadKind(kind), key, nonce, sealed.substr(0, kAeadTagBytes - 1), aad, &back),
            "short input accepted");
    }
  uint8_t hdr[80], out[32], out2[32];
  for (auto& b : hdr) b = uint8_t(rng());
  scrypt_1024_1_1(hdr, out);
  std::thread t([&] { scrypt_1024_1_1(hdr, out2); });  // per-thread scratch pad
  t.join();
  CHECK(std::memcmp(out, out2, 32) == 0, "scrypt differs across threads");
  // X11: first use races the one-time S-box / JH constant init across verifier threads.
  {
    uint8_t x[4][32];
    std::vector<std::thread> vs;
    for (int i = 0; i < 4; ++i) vs.emplace_back([&, i] { verify_share(Algo::kX11, hdr, hdr, x[i]); });
    for (auto& v : vs) v.join();
    for (int i = 1; i < 4; ++i) CHECK(std::memcmp(x[0], x[i], 32) == 0, "x11 differs across threads");
  }
  for (size_t kl : {0ul, 1ul, 64ul, 65ul, 200ul}) {
    std::vector<uint8_t> k(kl, 0x5a), msg(kl * 3 + 1, 0x33), dk(77);
    hmac_sha256(k.data(), k.size(), msg.data(), msg.size(), out);
    pbkdf2_sha256(k.data(), k.size(), msg.data(), msg.size(), 2, dk.data(), dk.size());
  }
}

int main(int argc, char** argv) {
  const double seconds = argc > 1 ? std::atof(argv[1]) : 4.0;
  test_share_queue();
  test_job_epochs(4, seconds);
  test_crypto_memory();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("runtime stress: all checks passed\n");
  return 0;
}
