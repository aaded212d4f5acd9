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
// Usage: proxlab LAYOUT [reps]   (LAYOUT: "numel nseg" then "offset numel" lines)
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

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: proxlab LAYOUT [reps]\n");
    return 2;
  }
  const int reps = argc > 2 ? atoi(argv[2]) : 50;
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
