// c_abi_round.cpp — a FedAvg aggregation round driven through the C ABI
// alone (include/fedagg.h; no Python, no torch): what a native FL server
// would call.  Builds N client buckets on the GPU, reduces them with
// fa_reduce (fused broadcast), and checks the result against a plain
// restatement of the reference order on the host:
//   - every tensor here has a column count that is a multiple of 32, so
//     every fp32 column takes the cascade order, which for N <= 16 clients is
//     the sequential sum from +0 (train_fedavg.py:145-146 via ATen's
//     multi_row_sum), then / N;
//   - the int64 scalar key (num_batches_tracked) takes .float(), the 8-lane
//     inner order for N >= 8, / N, and truncation toward zero.
// Exit status 0 = bit-exact.
//
// Build (done by feddct_amd/build.py):
//   hipcc --offload-arch=gfx950 -O2 -o examples/c_abi_round examples/c_abi_round.cpp \
//         -Iinclude -Lfeddct_amd -lfedagg -Wl,-rpath,<repo>/feddct_amd
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "fedagg.h"

#define CHECK_FA(x)                                                           \
  do {                                                                        \
    int rc_ = (x);                                                            \
    if (rc_ != FA_OK) {                                                       \
      fprintf(stderr, "%s -> %d: %s\n", #x, rc_, fa_last_error());           \
      return 2;                                                               \
    }                                                                         \
  } while (0)
#define CHECK_HIP(x)                                                          \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      return 2;                                                               \
    }                                                                         \
  } while (0)

// The 8-lane inner order of a single int64 column (n >= 8), as floats.
static float inner8(const std::vector<float>& x) {
  const int n = (int)x.size(), nv = n / 8;
  float fin = 0.f;
  for (int k = 8 * nv; k < n; ++k) fin += x[k];
  for (int l = 0; l < 8; ++l) {
    // ILP-4 over this lane's nv rows; with nv < 4 that is a plain sum into
    // partial 0 (nv / 4 == 0), then + 0 + 0 + 0
    float p[4] = {0.f, 0.f, 0.f, 0.f};
    const int q = nv / 4;
    for (int k = 0; k < 4; ++k)
      for (int r = 0; r < q; ++r) p[k] += x[l + 8 * (4 * r + k)];
    for (int r = 4 * q; r < nv; ++r) p[0] += x[l + 8 * r];
    fin += ((p[0] + p[1]) + p[2]) + p[3];
  }
  return fin;
}

int main() {
  printf("%s\n", fa_version());
  const int n = 12;                         // clients (slots)
  const int64_t sizes[] = {4096, 288, 64};  // fp32 tensors, multiples of 32
  std::vector<fa_seg> segs;
  int64_t off = 0;
  for (int64_t m : sizes) {
    segs.push_back(fa_seg{off, m});
    off += (m + 63) / 64 * 64;  // 256-B aligned tensors, as the arenas lay them out
  }
  const int64_t numel = off;
  fa_seg seg64{0, 1};

  // every client's bucket in ONE device allocation (a slab, as
  // feddct_amd/slab.py places them: separate allocations per client read up
  // to 8 % slower on some boxes)
  std::vector<float*> c32(n);
  std::vector<int64_t*> c64(n);
  float* slab32;
  int64_t* slab64;
  CHECK_HIP(hipMalloc(&slab32, (size_t)n * numel * sizeof(float)));
  CHECK_HIP(hipMalloc(&slab64, (size_t)n * sizeof(int64_t)));
  CHECK_HIP(hipMemset(slab32, 0, (size_t)n * numel * sizeof(float)));
  for (int i = 0; i < n; ++i) {
    c32[i] = slab32 + (size_t)i * numel;   // numel: a multiple of 64 floats (256 B)
    c64[i] = slab64 + i;
    for (size_t k = 0; k < segs.size(); ++k)
      CHECK_FA(fa_synth_fill_f32(c32[i] + segs[k].offset, segs[k].numel, (int)k, i, 0.f,
                                 0.05f, 1 /* adversarial: 2^+-20 dynamic range */, nullptr));
    CHECK_FA(fa_synth_fill_i64(c64[i], 1, 99, i, 0, nullptr));
  }
  float* g32;
  int64_t* g64;
  CHECK_HIP(hipMalloc(&g32, numel * sizeof(float)));
  CHECK_HIP(hipMalloc(&g64, sizeof(int64_t)));

  fa_plan* plan = nullptr;
  CHECK_FA(fa_plan_create(segs.data(), (int)segs.size(), numel, &seg64, 1, 1, 0,
                          FA_PLAN_GAPS_ARE_PADDING, &plan));
  fa_plan_info info;
  CHECK_FA(fa_plan_get_info(plan, &info));
  printf("plan: %d tiles (%d vector, %d scalar)\n", info.ntiles, info.ntiles_cascade,
         info.ntiles_tail);

  // host copies of the inputs, before the broadcast overwrites them
  std::vector<std::vector<float>> h32(n, std::vector<float>(numel));
  std::vector<int64_t> h64(n);
  for (int i = 0; i < n; ++i) {
    CHECK_HIP(hipMemcpy(h32[i].data(), c32[i], numel * sizeof(float), hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(&h64[i], c64[i], sizeof(int64_t), hipMemcpyDeviceToHost));
  }

  CHECK_FA(fa_reduce(plan, (const float* const*)c32.data(), (const int64_t* const*)c64.data(),
                     n, nullptr, g32, g64, FA_F_BCAST, nullptr));
  CHECK_HIP(hipDeviceSynchronize());

  std::vector<float> got(numel);
  int64_t got64;
  CHECK_HIP(hipMemcpy(got.data(), g32, numel * sizeof(float), hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(&got64, g64, sizeof(int64_t), hipMemcpyDeviceToHost));

  long bad = 0;
  volatile float fn = (float)n;
  for (const fa_seg& s : segs)
    for (int64_t e = s.offset; e < s.offset + s.numel; ++e) {
      volatile float acc = 0.f;
      for (int i = 0; i < n; ++i) acc = acc + h32[i][e];  // sequential, no FMA
      volatile float want = acc / fn;
      uint32_t a, b;
      float w = want;
      std::memcpy(&a, &got[e], 4);
      std::memcpy(&b, &w, 4);
      if (a != b && !(std::isnan(got[e]) && std::isnan(w))) ++bad;
    }
  std::vector<float> xi(n);
  for (int i = 0; i < n; ++i) xi[i] = (float)h64[i];
  const int64_t want64 = (int64_t)(inner8(xi) / fn);
  if (got64 != want64) ++bad;

  // the fused broadcast: every client bucket now holds the global state
  std::vector<float> back(numel);
  for (int i = 0; i < n && !bad; ++i) {
    CHECK_HIP(hipMemcpy(back.data(), c32[i], numel * sizeof(float), hipMemcpyDeviceToHost));
    for (const fa_seg& s : segs)
      if (std::memcmp(back.data() + s.offset, got.data() + s.offset, s.numel * 4)) ++bad;
  }

  CHECK_FA(fa_plan_destroy(plan));
  (void)hipFree(slab32);
  (void)hipFree(slab64);
  (void)hipFree(g32);
  (void)hipFree(g64);
  printf("%s: %ld mismatches over %ld fp32 + 1 int64 elements, broadcast checked\n",
         bad ? "FAIL" : "OK", bad, (long)(sizes[0] + sizes[1] + sizes[2]));
  return bad ? 1 : 0;
}
