// proxlab.hip — the FedProx proximal term's forward partial sums (csrc/prox.hip
// prox_partials) against the read ceiling, by chunking (r05, VERDICT r04
// next 4).  The product cuts every tensor into 4096-float chunks, one per
// workgroup: the wrn16_8 C100 layout's 2,690 chunks run 1.31 rounds of the
// chip's resident workgroups, so the last 0.31 round is a part-filled tail.
// Here, same process, same buffers (hashed data, 2 x 11.0 M floats):
//   fixed4096 / fixed2048 / fixed1024 : chunks of at most that many floats;
//   balanced_kR : a chunk size chosen so that the layout's chunk count fills
//                 exactly k rounds of this kernel's resident workgroups
//                 (<= k * slots), the size a multiple of 256 floats;
//   read_probe  : the same bytes read in the same shape, nothing computed
//                 (the ceiling);
// each with plain loads (the product's: the backward re-reads the buckets
// from the MALL) and nt loads.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/proxlab tools/proxlab.hip
// Usage: proxlab LAYOUT [reps] [step]   (LAYOUT: "numel nseg" then "offset numel" lines)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
struct Chunk {
  int64_t start;
  int32_t count;
  int32_t seg;
};
constexpr int kBlk = 256;

template <bool NT>
__device__ __forceinline__ f4 ld4(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// the product's kernel (CPW = 1), KV float4 per lane per bucket
template <int KV, bool NT, bool PROBE>
__global__ __launch_bounds__(kBlk) void partials(const Chunk* __restrict__ chunks,
                                                 const float* __restrict__ a,
                                                 const float* __restrict__ b,
                                                 float* __restrict__ out) {
  __shared__ float lds[kBlk / 64];
  const Chunk c = chunks[blockIdx.x];
  const int nv = c.count / 4;
  const f4* pa = reinterpret_cast<const f4*>(a + c.start);
  const f4* pb = reinterpret_cast<const f4*>(b + c.start);
  f4 xa[KV], xb[KV];
#pragma unroll
  for (int u = 0; u < KV; ++u) {
    const int v = threadIdx.x + u * kBlk;
    const bool ok = v < nv;
    xa[u] = ok ? ld4<NT>(pa + v) : f4{0.f, 0.f, 0.f, 0.f};
    xb[u] = ok ? ld4<NT>(pb + v) : f4{0.f, 0.f, 0.f, 0.f};
  }
  float acc = 0.f;
#pragma unroll
  for (int u = 0; u < KV; ++u) {
    if constexpr (PROBE) {
      const f4 s = xa[u] + xb[u];
      acc += s.x + s.y + s.z + s.w;
    } else {
      const f4 d = xa[u] - xb[u];
      acc += d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w;
    }
  }
  for (int j = 4 * nv + threadIdx.x; j < c.count; j += kBlk) {
    const float d = a[c.start + j] - b[c.start + j];
    acc += d * d;
  }
  acc = wave_sum(acc);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) lds[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float r = ((lds[0] + lds[1]) + lds[2]) + lds[3];
    if (!PROBE || r == 1234.5f) out[blockIdx.x] = r;
  }
}

// the product's backward (prox_grad<false,false>): g * (a - b) -> ga, -> gb;
// loads NTL, stores NTS
template <int KV, bool NTL, bool NTS>
__global__ __launch_bounds__(kBlk) void grad(const Chunk* __restrict__ chunks,
                                             const float* __restrict__ a,
                                             const float* __restrict__ b,
                                             const float* __restrict__ norms,
                                             float* __restrict__ ga, float* __restrict__ gb) {
  const Chunk c = chunks[blockIdx.x];
  const float nk = norms[c.seg];
  const float g = nk > 0.f ? 0.5f / nk : 0.f;
  const int nv = c.count / 4;
  const f4* pa = reinterpret_cast<const f4*>(a + c.start);
  const f4* pb = reinterpret_cast<const f4*>(b + c.start);
  f4* qa = reinterpret_cast<f4*>(ga + c.start);
  f4* qb = reinterpret_cast<f4*>(gb + c.start);
  f4 xa[KV], xb[KV];
#pragma unroll
  for (int u = 0; u < KV; ++u) {
    const int v = threadIdx.x + u * kBlk;
    const bool ok = v < nv;
    xa[u] = ok ? ld4<NTL>(pa + v) : f4{0.f, 0.f, 0.f, 0.f};
    xb[u] = ok ? ld4<NTL>(pb + v) : f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int u = 0; u < KV; ++u) {
    const int v = threadIdx.x + u * kBlk;
    if (v < nv) {
      const f4 d = g * (xa[u] - xb[u]);
      if constexpr (NTS) {
        __builtin_nontemporal_store(d, qa + v);
        __builtin_nontemporal_store(-d, qb + v);
      } else {
        qa[v] = d;
        qb[v] = -d;
      }
    }
  }
  for (int j = 4 * nv + threadIdx.x; j < c.count; j += kBlk) {
    const int64_t e = c.start + j;
    const float d = g * (a[e] - b[e]);
    ga[e] = d;
    gb[e] = -d;
  }
}

// the product's finish (LDS form): per tensor the partials -> sqrt -> norms,
// wave 0 sums the norms
__global__ __launch_bounds__(1024) void finish(const int* __restrict__ first, int nseg,
                                               int nchunks, const float* __restrict__ partials,
                                               float* __restrict__ norms,
                                               float* __restrict__ total) {
  extern __shared__ float dyn[];
  float* sp = dyn;
  int* sf = reinterpret_cast<int*>(dyn + nchunks);
  float* nl = reinterpret_cast<float*>(sf + nseg + 1);
  for (int j = threadIdx.x; j < nchunks; j += 1024) sp[j] = partials[j];
  for (int j = threadIdx.x; j <= nseg; j += 1024) sf[j] = first[j];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int k = wave; k < nseg; k += 16) {
    float sq = 0.f;
    for (int i = sf[k] + lane; i < sf[k + 1]; i += 64) sq += sp[i];
    sq = wave_sum(sq);
    if (lane == 0) nl[k] = norms[k] = sqrtf(sq);
  }
  __syncthreads();
  if (wave == 0) {
    float t = 0.f;
    for (int k = lane; k < nseg; k += 64) t += nl[k];
    t = wave_sum(t);
    if (lane == 0) *total = t;
  }
}

__global__ void hash_fill(float* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 0x9E3779B9u ^ seed;
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    p[i] = ((float)(int32_t)(h >> 8) - 8388608.0f) * (1.0f / 8388608.0f);
  }
}

std::vector<Chunk> cut(const std::vector<std::pair<int64_t, int64_t>>& segs, int64_t cs) {
  std::vector<Chunk> ch;
  for (size_t k = 0; k < segs.size(); ++k)
    for (int64_t c = 0; c < segs[k].second; c += cs)
      ch.push_back(Chunk{segs[k].first + c, (int32_t)std::min<int64_t>(cs, segs[k].second - c),
                         (int32_t)k});
  return ch;
}

template <int KV, bool NT, bool PROBE>
int slots_of() {
  int nb = 0, cus = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &nb, reinterpret_cast<const void*>(partials<KV, NT, PROBE>), kBlk, 0));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  return nb * cus;
}

template <int KV, bool NT, bool PROBE>
void launch(const Chunk* d, int n, const float* a, const float* b, float* out) {
  hipLaunchKernelGGL((partials<KV, NT, PROBE>), dim3(n), dim3(kBlk), 0, 0, d, a, b, out);
}

__global__ void read_flush(const f4* __restrict__ p, int64_t n, float* __restrict__ sink) {
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    acc += p[i];
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) sink[0] = 1.f;
}

// step mode (r05): the whole term per training step — partials, finish,
// grad — per MALL condition (below) before every step, per
// chunking x forward-load x backward-load x store policy; HIP events
// between the kernels
template <int KV>
void step_launch(const Chunk* d, int n, const int* first, int nseg, const float* a,
                 const float* b, float* part, float* norms, float* total, float* ga, float* gb,
                 bool ntf, bool ntl, bool nts, hipEvent_t* ev) {
  CK(hipEventRecord(ev[0], 0));
  if (ntf) hipLaunchKernelGGL((partials<KV, true, false>), dim3(n), dim3(kBlk), 0, 0, d, a, b, part);
  else hipLaunchKernelGGL((partials<KV, false, false>), dim3(n), dim3(kBlk), 0, 0, d, a, b, part);
  CK(hipEventRecord(ev[1], 0));
  hipLaunchKernelGGL(finish, dim3(1), dim3(1024), (size_t)(n + 2 * nseg + 1) * 4, 0, first, nseg,
                     n, part, norms, total);
  CK(hipEventRecord(ev[2], 0));
#define G(L, S) hipLaunchKernelGGL((grad<KV, L, S>), dim3(n), dim3(kBlk), 0, 0, d, a, b, norms, ga, gb)
  if (ntl) {
    if (nts) G(true, true);
    else G(true, false);
  } else {
    if (nts) G(false, true);
    else G(false, false);
  }
#undef G
  CK(hipEventRecord(ev[3], 0));
}

int run_steps(const std::vector<std::pair<int64_t, int64_t>>& segs, int64_t elems, long long numel,
              const float* a, const float* b, float* out, int s4, int s2, int s1, int reps) {
  (void)out;
  float *ga, *gb, *part, *norms, *total, *flush;
  CK(hipMalloc(&ga, numel * 4));
  CK(hipMalloc(&gb, numel * 4));
  CK(hipMalloc(&part, 64 << 20));
  CK(hipMalloc(&norms, segs.size() * 4 + 4));
  CK(hipMalloc(&total, 16));
  const size_t fl = (size_t)1 << 30;
  CK(hipMalloc(&flush, fl));
  struct C {
    std::string name;
    int64_t cs;
    int kv;
  };
  std::vector<C> cuts = {{"fixed4096", 4096, 4}, {"fixed2048", 2048, 2}};
  for (int64_t cs = 256; cs <= 4096; cs += 256) {
    const int kv = (int)((cs + 1023) / 1024);
    const int s = kv >= 3 ? s4 : kv == 2 ? s2 : s1;
    if ((int64_t)cut(segs, cs).size() <= 4LL * s) {
      cuts.push_back({"balanced_4R", cs, kv == 3 ? 4 : kv});
      break;
    }
  }
  const double fwd = 8.0 * elems, bwd = 16.0 * elems;
  std::vector<hipEvent_t> evs((size_t)reps * 4);
  for (auto& e : evs) CK(hipEventCreate(&e));
  for (int pass = 0; pass < 3; ++pass)
    for (const C& c : cuts) {
      const std::vector<Chunk> ch = cut(segs, c.cs);
      std::vector<int> first(segs.size() + 1, 0);  // per segment its first chunk
      for (const Chunk& x : ch) ++first[x.seg + 1];
      for (size_t k = 0; k < segs.size(); ++k) first[k + 1] += first[k];
      Chunk* d;
      int* df;
      CK(hipMalloc(&d, ch.size() * sizeof(Chunk)));
      CK(hipMalloc(&df, first.size() * sizeof(int)));
      CK(hipMemcpy(d, ch.data(), ch.size() * sizeof(Chunk), hipMemcpyHostToDevice));
      CK(hipMemcpy(df, first.data(), first.size() * sizeof(int), hipMemcpyHostToDevice));
      const int n = (int)ch.size(), nseg = (int)segs.size();
      for (int fm = 0; fm < 3; ++fm)
      for (int pol = 0; pol < 8; ++pol) {
        const bool ntf = pol & 1, ntl = pol & 2, nts = pol & 4;
        for (int r = -2; r < reps; ++r) {
          // flush: 0 none (back-to-back steps, the bench's condition), 1 a
          // 1 GiB plain read (the MALL holds clean other lines), 2 a 1 GiB
          // memset (dirty other lines)
          if (fm == 2) CK(hipMemsetAsync(flush, r & 0xff, fl, 0));
          if (fm == 1)
            hipLaunchKernelGGL(read_flush, dim3(4096), dim3(256), 0, 0,
                               reinterpret_cast<const f4*>(flush), (int64_t)(fl / 16), total + 2);
          hipEvent_t* ev = &evs[(size_t)std::max(r, 0) * 4];
          if (c.kv == 4) step_launch<4>(d, n, df, nseg, a, b, part, norms, total, ga, gb, ntf, ntl, nts, ev);
          else if (c.kv == 2) step_launch<2>(d, n, df, nseg, a, b, part, norms, total, ga, gb, ntf, ntl, nts, ev);
          else step_launch<1>(d, n, df, nseg, a, b, part, norms, total, ga, gb, ntf, ntl, nts, ev);
        }
        CK(hipDeviceSynchronize());
        std::vector<float> tp, tf, tg, tt;
        for (int r = 0; r < reps; ++r) {
          float x[3];
          for (int i = 0; i < 3; ++i) CK(hipEventElapsedTime(&x[i], evs[r * 4 + i], evs[r * 4 + i + 1]));
          tp.push_back(x[0] * 1e3f);
          tf.push_back(x[1] * 1e3f);
          tg.push_back(x[2] * 1e3f);
          tt.push_back((x[0] + x[1] + x[2]) * 1e3f);
        }
        auto med = [](std::vector<float> v) {
          std::sort(v.begin(), v.end());
          return (double)v[v.size() / 2];
        };
        printf("{\"exp\": \"proxlab_step\", \"flush\": %d, \"pass\": %d, \"cut\": \"%s\", \"chunk\": %lld, "
               "\"chunks\": %d, \"fwd_nt\": %d, \"bwd_nt_loads\": %d, \"bwd_nt_stores\": %d, "
               "\"partials_us\": %.2f, \"finish_us\": %.2f, \"grad_us\": %.2f, \"step_us\": %.2f, "
               "\"frac\": %.4f}\n",
               fm, pass, c.name.c_str(), (long long)c.cs, n, (int)ntf, (int)ntl, (int)nts, med(tp),
               med(tf), med(tg), med(tt), (fwd + bwd) / (med(tt) * 1e-6) / 8e12);
        fflush(stdout);
      }
      CK(hipFree(d));
      CK(hipFree(df));
    }
  CK(hipGetLastError());
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: proxlab LAYOUT [reps]\n");
    return 2;
  }
  const int reps = argc > 2 ? atoi(argv[2]) : 50;
  const bool step_mode = argc > 3 && strcmp(argv[3], "step") == 0;
  FILE* f = fopen(argv[1], "r");
  long long numel;
  int nseg;
  if (!f || fscanf(f, "%lld %d", &numel, &nseg) != 2) return 2;
  std::vector<std::pair<int64_t, int64_t>> segs(nseg);
  int64_t elems = 0;
  for (auto& s : segs) {
    long long o, m;
    if (fscanf(f, "%lld %lld", &o, &m) != 2) return 2;
    s = {o, m};
    elems += m;
  }
  fclose(f);
  float *a, *b, *out;
  CK(hipMalloc(&a, numel * 4));
  CK(hipMalloc(&b, numel * 4));
  CK(hipMalloc(&out, 1 << 22));
  hipLaunchKernelGGL(hash_fill, dim3(4096), dim3(256), 0, 0, a, (int64_t)numel, 1u);
  hipLaunchKernelGGL(hash_fill, dim3(4096), dim3(256), 0, 0, b, (int64_t)numel, 2u);
  const int s4 = slots_of<4, false, false>(), s2 = slots_of<2, false, false>(),
            s1 = slots_of<1, false, false>();
  struct V {
    std::string name;
    int64_t cs;
    int kv;
    bool nt, probe;
  };
  std::vector<V> vs;
  for (int nt = 0; nt < 2; ++nt) {
    const char* sfx = nt ? "_nt" : "";
    vs.push_back({std::string("fixed4096") + sfx, 4096, 4, nt != 0, false});
    vs.push_back({std::string("fixed2048") + sfx, 2048, 2, nt != 0, false});
    vs.push_back({std::string("fixed1024") + sfx, 1024, 1, nt != 0, false});
    vs.push_back({std::string("probe4096") + sfx, 4096, 4, nt != 0, true});
    // balanced: the smallest 256-multiple chunk with count <= k * slots
    for (int k = 1; k <= 4; ++k) {
      for (int64_t cs = 256; cs <= 4096; cs += 256) {
        const int kv = (int)((cs + 1023) / 1024);
        const int s = kv == 4 || kv == 3 ? s4 : kv == 2 ? s2 : s1;
        const int64_t n = (int64_t)cut(segs, cs).size();
        if (n <= (int64_t)k * s) {
          vs.push_back({"balanced_" + std::to_string(k) + "R" + sfx, cs, kv == 3 ? 4 : kv,
                        nt != 0, false});
          break;
        }
      }
    }
  }
  if (step_mode) return run_steps(segs, elems, numel, a, b, out, s4, s2, s1, reps);
  std::vector<Chunk*> dch(vs.size());
  std::vector<int> nch(vs.size());
  for (size_t i = 0; i < vs.size(); ++i) {
    const std::vector<Chunk> c = cut(segs, vs[i].cs);
    nch[i] = (int)c.size();
    CK(hipMalloc(&dch[i], c.size() * sizeof(Chunk)));
    CK(hipMemcpy(dch[i], c.data(), c.size() * sizeof(Chunk), hipMemcpyHostToDevice));
  }
  auto run = [&](size_t i) {
    const V& v = vs[i];
#define L(KV)                                                                   \
  do {                                                                          \
    if (v.probe) {                                                              \
      if (v.nt) launch<KV, true, true>(dch[i], nch[i], a, b, out);              \
      else launch<KV, false, true>(dch[i], nch[i], a, b, out);                  \
    } else {                                                                    \
      if (v.nt) launch<KV, true, false>(dch[i], nch[i], a, b, out);             \
      else launch<KV, false, false>(dch[i], nch[i], a, b, out);                 \
    }                                                                           \
  } while (0)
    if (v.kv == 4) L(4);
    else if (v.kv == 2) L(2);
    else L(1);
#undef L
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ts(vs.size());
  for (int pass = 0; pass < 7; ++pass)
    for (size_t i = 0; i < vs.size(); ++i) {
      for (int w = 0; w < 3; ++w) run(i);
      CK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r) run(i);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts[i].push_back(ms * 1e3f / reps);
    }
  CK(hipGetLastError());
  const double bytes = 8.0 * elems;
  for (size_t i = 0; i < vs.size(); ++i) {
    std::vector<float> t = ts[i];
    std::sort(t.begin(), t.end());
    const double us = t[t.size() / 2];
    const int s = vs[i].kv == 4 ? s4 : vs[i].kv == 2 ? s2 : s1;
    printf("{\"exp\": \"proxlab\", \"variant\": \"%s\", \"chunk\": %lld, \"chunks\": %d, "
           "\"slots\": %d, \"rounds\": %.3f, \"us_median\": %.2f, \"us_min\": %.2f, "
           "\"bytes\": %.0f, \"TBps\": %.3f}\n",
           vs[i].name.c_str(), (long long)vs[i].cs, nch[i], s, (double)nch[i] / s, us,
           (double)t[0], bytes, bytes / (us * 1e-6) / 1e12);
  }
  return 0;
}
