// loop_round.cpp — TEST DRIVER: the native multi-rank rounds of
// libfedagg_comm (chained, striped, sharded with either e1 exchange) run with
// W ranks on one GPU over the loopback communicator (loopccl.hip), checked
// against one GPU's fa_reduce over all clients:
//   chained / striped / blocked / multi / mean_multi: bit-identical (fp32 and
//   int64; mean_multi has no int64 keys);
//   sharded / multi_e1 (e1): int64 bit-identical, fp32 within the forward
//   error bound of two N-term sums, 2N * 2^-24 * sum_i |w_i x_i| (any
//   summation order).
// Usage: loop_round LAYOUT CASE...
//   LAYOUT: "f32_numel i64_numel nseg32 nseg64 [P]" then one "offset numel"
//           line per segment (fp32 first), as BucketLayout.segs32 / segs64;
//           with P, fp32 lines are "offset numel key mu sigma" and int64
//           lines "offset numel key": the digest generator's per-key
//           parameters (feddct_amd/workload.py fill_client), so a result can
//           be checked against tests/golden/digests.json (FA_LOOP_DUMP).
//   CASE:   mode:W:counts:root:model:weighted:nchunks
//           mode   chained | striped | blocked | sharded | sharded_rs
//                  | multi (the default entry: fa_multi_plan_create /
//                    fa_reduce_multi) | multi_e1 (FA_MULTI_REASSOCIATE)
//                  | mean_multi (fa_mean_f32_multi: fp32 keys only)
//           counts comma-separated client slots per rank (sum = N)
//           root   result rank, or -1 for every rank
//           model  threads (one thread + comm per rank: fa_comm_init_rank)
//                  | single (one thread drives all ranks: fa_comm_init; only
//                    for schedules whose p2p pairs share a step: sharded, blocked)
// One JSON line per case; exit status 0 iff every case passed.
// FA_LOOP_DUMP=path: the first result rank's out32 then out64, raw, of the
// last case.
// FA_LOOP_PROFILE=1 (threads model): every rank's communicator profiles its
// round (fa_comm_set_profile) and the line carries rank 0's
// fa_round_plan_profile.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "fedagg.h"
#include "fedagg_comm.h"

namespace {

struct Layout {
  int64_t f32_numel = 0, i64_numel = 0;
  std::vector<fa_seg> s32, s64;
  bool params = false;                 // per-key generator parameters given
  std::vector<int> key32, key64;
  std::vector<float> mu, sigma;
};

struct Case {
  std::string mode, model, text;
  int W = 0, root = -1, weighted = 0, nchunks = 0;
  std::vector<int> counts;
};

bool read_layout(const char* path, Layout* L) {
  FILE* f = fopen(path, "r");
  if (!f) return false;
  char line[256];
  long long a, b;
  int n32, n64;
  char tag[8] = {0};
  if (!fgets(line, sizeof line, f)) return false;
  const int got = sscanf(line, "%lld %lld %d %d %7s", &a, &b, &n32, &n64, tag);
  if (got < 4) return false;
  L->params = got == 5 && tag[0] == 'P';
  L->f32_numel = a;
  L->i64_numel = b;
  for (int i = 0; i < n32 + n64; ++i) {
    long long o, m;
    if (fscanf(f, "%lld %lld", &o, &m) != 2) return false;
    (i < n32 ? L->s32 : L->s64).push_back(fa_seg{o, m});
    if (!L->params) continue;
    int k;
    if (fscanf(f, "%d", &k) != 1) return false;
    if (i < n32) {
      float mu, sg;
      if (fscanf(f, "%f %f", &mu, &sg) != 2) return false;
      L->key32.push_back(k);
      L->mu.push_back(mu);
      L->sigma.push_back(sg);
    } else {
      L->key64.push_back(k);
    }
  }
  fclose(f);
  return true;
}

bool parse_case(const std::string& s, Case* c) {
  std::vector<std::string> f;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ':')) f.push_back(tok);
  if (f.size() != 7) return false;
  c->text = s;
  c->mode = f[0];
  c->W = atoi(f[1].c_str());
  std::stringstream cs(f[2]);
  while (std::getline(cs, tok, ',')) c->counts.push_back(atoi(tok.c_str()));
  c->root = atoi(f[3].c_str());
  c->model = f[4];
  c->weighted = atoi(f[5].c_str());
  c->nchunks = atoi(f[6].c_str());
  return (int)c->counts.size() == c->W;
}

#define HIPC(x)                                                             \
  do {                                                                      \
    if ((x) != hipSuccess) {                                                \
      fprintf(stderr, "%s failed\n", #x);                                   \
      exit(2);                                                              \
    }                                                                       \
  } while (0)

struct Rank {
  fa_comm* comm = nullptr;
  void* plan = nullptr;
  hipStream_t st = nullptr;
  fa_shard_io io{};
  std::vector<const float*> c32;
  std::vector<const int64_t*> c64;
  int rc = 0;
  std::string err;
  fa_round_profile prof{};
  bool has_prof = false;
};

int create_plan(const Case& c, const Layout& L, Rank& r) {
  const unsigned fl = FA_PLAN_GAPS_ARE_PADDING;
  const fa_seg* s64 = L.s64.empty() ? nullptr : L.s64.data();
  if (c.mode == "mean_multi") return 0;  // stateless: cached in the communicator
  if (c.mode == "multi" || c.mode == "multi_e1")
    return fa_multi_plan_create(r.comm, L.s32.data(), (int)L.s32.size(), L.f32_numel, s64,
                                (int)L.s64.size(), L.i64_numel, c.counts.data(), c.nchunks, fl,
                                c.mode == "multi" ? FA_MULTI_EXACT : FA_MULTI_REASSOCIATE,
                                (fa_multi_plan**)&r.plan);
  if (c.mode == "chained")
    return fa_chain_plan_create(r.comm, L.s32.data(), (int)L.s32.size(), L.f32_numel, s64,
                                (int)L.s64.size(), L.i64_numel, c.counts.data(), c.nchunks, fl,
                                (fa_chain_plan**)&r.plan);
  if (c.mode == "striped")
    return fa_stripe_plan_create_ex(r.comm, L.s32.data(), (int)L.s32.size(), L.f32_numel, s64,
                                    (int)L.s64.size(), L.i64_numel, c.counts.data(), c.nchunks,
                                    fl, (fa_stripe_plan**)&r.plan);
  if (c.mode == "blocked")
    return fa_block_plan_create(r.comm, L.s32.data(), (int)L.s32.size(), L.f32_numel, s64,
                                (int)L.s64.size(), L.i64_numel, c.counts.data(), fl,
                                (fa_block_plan**)&r.plan);
  return fa_shard_plan_create_ex(r.comm, L.s32.data(), (int)L.s32.size(), L.f32_numel, s64,
                                 (int)L.s64.size(), L.i64_numel, c.counts.data(), c.nchunks,
                                 c.mode == "sharded_rs" ? FA_XCHG_RS_GATHER : FA_XCHG_REDUCE, fl,
                                 (fa_shard_plan**)&r.plan);
}

int run_round(const Case& c, const Layout& L, std::vector<Rank*>& ranks,
              std::vector<void*>& plans, std::vector<fa_shard_io>& io) {
  const int nl = (int)plans.size();
  if (c.mode == "mean_multi") {
    if (nl != 1) return -1;  // one thread per rank only
    return fa_mean_f32_multi(ranks[0]->comm, io[0].c32, c.counts.data(), L.f32_numel,
                             io[0].out32, L.s32.data(), (int)L.s32.size(), c.root, io[0].stream);
  }
  if (c.mode == "multi" || c.mode == "multi_e1")
    return fa_reduce_multi((fa_multi_plan* const*)plans.data(), nl, io.data(), c.root);
  if (c.mode == "chained")
    return fa_reduce_chained((fa_chain_plan* const*)plans.data(), nl, io.data(), c.root);
  if (c.mode == "striped")
    return fa_reduce_striped((fa_stripe_plan* const*)plans.data(), nl, io.data(), c.root);
  if (c.mode == "blocked")
    return fa_reduce_blocked((fa_block_plan* const*)plans.data(), nl, io.data(), c.root);
  return fa_reduce_sharded((fa_shard_plan* const*)plans.data(), nl, io.data(), c.root);
}

void destroy_plan(const Case& c, void* p) {
  if (!p) return;
  if (c.mode == "multi" || c.mode == "multi_e1") {
    fa_multi_plan_destroy((fa_multi_plan*)p);
    return;
  }
  if (c.mode == "chained") fa_chain_plan_destroy((fa_chain_plan*)p);
  else if (c.mode == "striped") fa_stripe_plan_destroy((fa_stripe_plan*)p);
  else if (c.mode == "blocked") fa_block_plan_destroy((fa_block_plan*)p);
  else fa_shard_plan_destroy((fa_shard_plan*)p);
}

bool run_case(const Case& c, const Layout& L) {
  int n = 0;
  for (int k : c.counts) n += k;
  const int64_t F = L.f32_numel, I = std::max<int64_t>(L.i64_numel, 1);
  // clients: the portable synthetic state, one seed per slot
  std::vector<float*> c32(n);
  std::vector<int64_t*> c64(n);
  for (int i = 0; i < n; ++i) {
    HIPC(hipMalloc(&c32[i], F * 4));
    HIPC(hipMalloc(&c64[i], I * 8));
    HIPC(hipMemset(c32[i], 0, F * 4));
    HIPC(hipMemset(c64[i], 0, I * 8));
    for (size_t k = 0; k < L.s32.size(); ++k)
      fa_synth_fill_f32(c32[i] + L.s32[k].offset, L.s32[k].numel,
                        L.params ? L.key32[k] : (int)k, i, L.params ? L.mu[k] : 0.f,
                        L.params ? L.sigma[k] : 0.05f, 0, nullptr);
    for (size_t k = 0; k < L.s64.size(); ++k)
      fa_synth_fill_i64(c64[i] + L.s64[k].offset, L.s64[k].numel,
                        L.params ? L.key64[k] : (int)(1000 + k), i, 0, nullptr);
  }
  std::vector<float> w(n);
  double ws = 0;
  for (int i = 0; i < n; ++i) ws += i + 1;
  for (int i = 0; i < n; ++i) w[i] = (float)((i + 1) / ws);
  float* dw = nullptr;
  HIPC(hipMalloc(&dw, n * 4));
  HIPC(hipMemcpy(dw, w.data(), n * 4, hipMemcpyHostToDevice));

  // the single-GPU reference
  float* ref32;
  int64_t* ref64;
  HIPC(hipMalloc(&ref32, F * 4));
  HIPC(hipMalloc(&ref64, I * 8));
  HIPC(hipMemset(ref32, 0, F * 4));
  HIPC(hipMemset(ref64, 0, I * 8));
  fa_plan* rp = nullptr;
  const fa_seg* s64 = L.s64.empty() ? nullptr : L.s64.data();
  int rc = fa_plan_create(L.s32.data(), (int)L.s32.size(), F, s64, (int)L.s64.size(),
                          L.i64_numel, 0, FA_PLAN_GAPS_ARE_PADDING, &rp);
  if (!rc)
    rc = fa_reduce(rp, (const float* const*)c32.data(), (const int64_t* const*)c64.data(), n,
                   c.weighted ? dw : nullptr, ref32, ref64, 0, nullptr);
  HIPC(hipDeviceSynchronize());
  if (rc) {
    printf("{\"case\": \"%s\", \"ok\": false, \"error\": \"reference: %s\"}\n", c.text.c_str(),
           fa_last_error());
    return false;
  }
  fa_plan_destroy(rp);

  // the ranks
  const int W = c.W;
  std::vector<Rank> R(W);
  std::vector<float*> out32(W, nullptr);
  std::vector<int64_t*> out64(W, nullptr);
  int slot = 0;
  for (int r = 0; r < W; ++r) {
    const bool result = c.root < 0 || c.root == r;
    if (result) {
      HIPC(hipMalloc(&out32[r], F * 4));
      HIPC(hipMalloc(&out64[r], I * 8));
      HIPC(hipMemset(out32[r], 0xFF, F * 4));  // NaN fill: an unwritten element fails
      HIPC(hipMemset(out64[r], 0xFF, I * 8));
    }
    for (int j = 0; j < c.counts[r]; ++j) {
      R[r].c32.push_back(c32[slot + j]);
      R[r].c64.push_back(c64[slot + j]);
    }
    R[r].io.c32 = R[r].c32.data();
    R[r].io.c64 = L.s64.empty() ? nullptr : R[r].c64.data();
    R[r].io.weights = c.weighted ? dw + slot : nullptr;
    R[r].io.out32 = out32[r];
    R[r].io.out64 = out64[r];
    slot += c.counts[r];
  }
  std::string err;
  bool failed = false;
  if (c.model == "threads") {
    unsigned char uid[FA_COMM_UID_BYTES];
    if (fa_comm_unique_id(uid, FA_COMM_UID_BYTES)) {
      err = fa_last_error();
      failed = true;
    } else {
      std::vector<std::thread> th;
      for (int r = 0; r < W; ++r)
        th.emplace_back([&, r] {
          Rank& k = R[r];
          (void)hipSetDevice(0);
          k.rc = fa_comm_init_rank(W, r, uid, FA_COMM_UID_BYTES, &k.comm);
          // the loopback pairs sends and receives on the host: never captured
          if (!k.rc) k.rc = fa_comm_set_graphs(k.comm, 0);
          const bool prof = getenv("FA_LOOP_PROFILE") && atoi(getenv("FA_LOOP_PROFILE"));
          if (!k.rc && prof) k.rc = fa_comm_set_profile(k.comm, 1);
          if (!k.rc) k.rc = create_plan(c, L, k);
          if (!k.rc) k.rc = hipStreamCreate(&k.st) == hipSuccess ? 0 : -1;
          if (!k.rc) {
            k.io.stream = k.st;
            std::vector<void*> plans{k.plan};
            std::vector<fa_shard_io> io{k.io};
            std::vector<Rank*> rk{&k};
            k.rc = run_round(c, L, rk, plans, io);
            if (!k.rc && prof && k.plan) {
              k.rc = fa_round_plan_profile(k.plan, &k.prof);
              k.has_prof = k.rc == 0;
            }
          }
          if (k.rc) k.err = fa_last_error();
          if (k.st) (void)hipStreamSynchronize(k.st);
        });
      for (auto& t : th) t.join();
    }
  } else {
    std::vector<fa_comm*> comms(W, nullptr);
    std::vector<int> devs(W, 0);
    rc = fa_comm_init(W, devs.data(), comms.data());
    if (rc) {
      err = fa_last_error();
      failed = true;
    } else {
      std::vector<void*> plans(W);
      std::vector<fa_shard_io> io(W);
      std::vector<Rank*> rk(W);
      for (int r = 0; r < W && !failed; ++r) {
        R[r].comm = comms[r];
        R[r].rc = create_plan(c, L, R[r]);
        HIPC(hipStreamCreate(&R[r].st));
        R[r].io.stream = R[r].st;
        plans[r] = R[r].plan;
        io[r] = R[r].io;
        rk[r] = &R[r];
        if (R[r].rc) {
          R[r].err = fa_last_error();
          failed = true;
        }
      }
      if (!failed) {
        rc = run_round(c, L, rk, plans, io);
        if (rc) {
          err = fa_last_error();
          failed = true;
        }
      }
    }
  }
  HIPC(hipDeviceSynchronize());
  for (int r = 0; r < W; ++r)
    if (R[r].rc) {
      failed = true;
      if (err.empty()) err = "rank " + std::to_string(r) + ": " + R[r].err;
    }

  // compare
  std::vector<float> ref(F), got(F);
  std::vector<int64_t> ref_i(I), got_i(I);
  HIPC(hipMemcpy(ref.data(), ref32, F * 4, hipMemcpyDeviceToHost));
  HIPC(hipMemcpy(ref_i.data(), ref64, I * 8, hipMemcpyDeviceToHost));
  const bool exact = c.mode == "chained" || c.mode == "striped" || c.mode == "blocked" ||
                     c.mode == "multi" || c.mode == "mean_multi";
  const bool with64 = c.mode != "mean_multi";
  std::vector<double> bound;
  if (!exact && !failed) {
    // forward error bound: 2N * 2^-24 * sum |w_i x_i| (/N for the mean)
    bound.assign(F, 0.0);
    std::vector<float> x(F);
    for (int i = 0; i < n; ++i) {
      HIPC(hipMemcpy(x.data(), c32[i], F * 4, hipMemcpyDeviceToHost));
      const double wi = c.weighted ? (double)w[i] : 1.0 / n;
      for (int64_t e = 0; e < F; ++e) bound[e] += std::fabs((double)x[e]) * wi;
    }
    for (int64_t e = 0; e < F; ++e) bound[e] = bound[e] * 2.0 * n * std::ldexp(1.0, -24) + 1e-38;
  }
  long long bad32 = 0, bad64 = 0, checked = 0;
  double worst = 0.0;
  std::string where;  // per failing rank: count, first / last bad element, unwritten (NaN)
  for (int r = 0; r < W && !failed; ++r) {
    if (!out32[r]) continue;
    HIPC(hipMemcpy(got.data(), out32[r], F * 4, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(got_i.data(), out64[r], I * 8, hipMemcpyDeviceToHost));
    ++checked;
    long long rb = 0, nan = 0;
    int64_t first = -1, last = -1;
    for (const fa_seg& s : L.s32)
      for (int64_t e = s.offset; e < s.offset + s.numel; ++e) {
        bool b;
        if (exact) {
          b = memcmp(&got[e], &ref[e], 4) != 0;
        } else {
          const double d = std::fabs((double)got[e] - (double)ref[e]);
          b = !(d <= bound[e]);
          if (d / bound[e] > worst) worst = d / bound[e];
        }
        if (b) {
          ++rb;
          if (std::isnan(got[e])) ++nan;
          if (first < 0) first = e;
          last = e;
        }
      }
    bad32 += rb;
    if (rb)
      where += "rank " + std::to_string(r) + ": " + std::to_string(rb) + " bad in [" +
               std::to_string(first) + ", " + std::to_string(last) + "], " +
               std::to_string(nan) + " unwritten; ";
    for (const fa_seg& s : L.s64)
      for (int64_t e = s.offset; e < s.offset + s.numel && with64; ++e)
        if (got_i[e] != ref_i[e]) ++bad64;
    const char* dump = getenv("FA_LOOP_DUMP");
    if (dump && checked == 1) {
      FILE* df = fopen(dump, "wb");
      if (df) {
        fwrite(got.data(), 4, (size_t)F, df);
        fwrite(got_i.data(), 8, (size_t)I, df);
        fclose(df);
      }
    }
  }
  const bool ok = !failed && bad32 == 0 && bad64 == 0 && checked > 0;
  if (err.empty()) err = where;
  char pbuf[256] = "null";
  if (R[0].has_prof)
    snprintf(pbuf, sizeof pbuf,
             "{\"exchange_us\": %.2f, \"comm_kernel_us\": %.2f, \"compute_kernel_us\": %.2f, "
             "\"wall_us\": %.2f, \"groups\": %d, \"kernels\": %d}",
             R[0].prof.exchange_us, R[0].prof.comm_kernel_us, R[0].prof.compute_kernel_us,
             R[0].prof.wall_us, R[0].prof.groups, R[0].prof.kernels);
  printf("{\"case\": \"%s\", \"ok\": %s, \"n\": %d, \"result_ranks\": %lld, \"bad_f32\": %lld, "
         "\"bad_i64\": %lld, \"check\": \"%s\", \"worst_err_over_bound\": %.4g, \"error\": \"%s\", "
         "\"profile\": %s}\n",
         c.text.c_str(), ok ? "true" : "false", n, checked, bad32, bad64,
         exact ? "bit-exact" : "error bound", worst, err.c_str(), pbuf);
  fflush(stdout);

  for (int r = 0; r < W; ++r) {
    destroy_plan(c, R[r].plan);
    if (R[r].st) (void)hipStreamDestroy(R[r].st);
    if (R[r].comm) fa_comm_destroy(R[r].comm);
    if (out32[r]) (void)hipFree(out32[r]);
    if (out64[r]) (void)hipFree(out64[r]);
  }
  for (int i = 0; i < n; ++i) {
    (void)hipFree(c32[i]);
    (void)hipFree(c64[i]);
  }
  (void)hipFree(ref32);
  (void)hipFree(ref64);
  (void)hipFree(dw);
  return ok;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: loop_round LAYOUT CASE...\n");
    return 2;
  }
  Layout L;
  if (!read_layout(argv[1], &L)) {
    fprintf(stderr, "bad layout file %s\n", argv[1]);
    return 2;
  }
  int fails = 0;
  for (int a = 2; a < argc; ++a) {
    Case c;
    if (!parse_case(argv[a], &c)) {
      fprintf(stderr, "bad case %s\n", argv[a]);
      return 2;
    }
    if (!run_case(c, L)) ++fails;
  }
  return fails ? 1 : 0;
}
