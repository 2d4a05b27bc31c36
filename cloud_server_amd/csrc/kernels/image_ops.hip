// Batched image-preprocessing kernels (gfx950 / CDNA4) over uint8 [N, H, W] batches.
//
// Reference: apps/preprocess/preprocess.py:18-227 runs one OpenCV call per image per op
// on the CPU, re-reading and re-writing a JPEG every time (views.py:95-137).  Here the
// whole labelled set lives on the device as one uint8 tensor and each op is one launch
// over the batch.  Numerics follow the spec'd NumPy reference (preprocess/ops_ref.py):
// border modes REFLECT_101 (linear filters, CLAHE padding, NL-means), REPLICATE
// (median, resize), "ignore outside" (erode/dilate); rounding = rint (half-even) then
// saturate, done in double where the reference rounds a double, so results are
// bit-identical except NL-means/resize (float exp / tap order: |diff| <= 1).
//
// Layout: most ops use one workgroup (256 threads = 4 waves) per image, the image
// staged once in LDS; 28x28 digit batches give N workgroups, so a 1k-image batch
// already fills all 256 CUs several times over.  Elementwise ops are grid-stride.
#include "common.h"

// Bit-parity with the NumPy reference: no FMA contraction of the double arithmetic here
// (the library is built with -ffp-contract=fast-honor-pragmas for the training kernels).
#pragma clang fp contract(off)

namespace csa {

constexpr int IMG_THREADS = 256;
constexpr int MAX_IMG_PIX = 128 * 128;       // LDS-resident image limit (H*W)

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}
__device__ __forceinline__ int clampi(int i, int n) { return i < 0 ? 0 : (i >= n ? n - 1 : i); }
__device__ __forceinline__ uint8_t sat_rint(double v) {
  v = rint(v);
  return (uint8_t)(v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v));
}

// ------------------------------------------------------------------ counter RNG
// Counter-based draws shared bit for bit with ops_ref.crng (NumPy): image i, draw j ->
// splitmix64(splitmix64((i << 32) | j) ^ seed) >> 32.  No state: every pixel/thread
// computes its own draw, so the random ops run entirely on the device.
__device__ __forceinline__ uint64_t smix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint32_t crng(uint64_t seed, uint64_t i, uint64_t j) {
  return (uint32_t)(smix(smix((i << 32) | j) ^ seed) >> 32);
}
__device__ __forceinline__ double crng_uniform(uint64_t seed, uint64_t i, uint64_t j) {   // [0, 1), 24 bits
  return (double)(crng(seed, i, j) >> 8) * (1.0 / 16777216.0);
}
__device__ __forceinline__ int crng_below(uint64_t seed, uint64_t i, uint64_t j, uint32_t n) {   // [0, n)
  return (int)(((uint64_t)crng(seed, i, j) * n) >> 32);
}

// ------------------------------------------------------------------ flips (P0-P2)
// mode 0: up-down, 1: left-right, 2: both (the reference "transpose" = cv2.flip(-1))
__global__ __launch_bounds__(256) void flip_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                   long total, int H, int W, int mode) {
  const long HW = (long)H * W;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / HW;
    const int r = (int)(i - n * HW);
    const int y = r / W, x = r - (r / W) * W;
    const int sy = (mode == 1) ? y : H - 1 - y;
    const int sx = (mode == 0) ? x : W - 1 - x;
    out[i] = in[n * HW + (long)sy * W + sx];
  }
}

// ------------------------------------------------------------------ affine intensity (P3/P4)
// y = x * alpha[n] + beta[n]; saturate (rint+clip) or wrap (trunc mod 256, numpy uint8
// element assignment in the reference loop).  Per-image alpha/beta let the random
// variant draw on the host with the reference RNG call order.
__global__ __launch_bounds__(256) void affine_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                     long total, long HW, const double* __restrict__ alpha,
                                                     const double* __restrict__ beta, int wrap) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / HW;
    const double v = (double)in[i] * alpha[n] + beta[n];
    if (wrap) {
      long t = (long)trunc(v) % 256;
      out[i] = (uint8_t)(t < 0 ? t + 256 : t);
    } else {
      out[i] = sat_rint(v);
    }
  }
}

// random variant: alpha = U(0, max_alpha), beta = randint(-max_beta, max_beta) per image
// from the counter RNG (draws 0 and 1 of image n), computed by every thread itself
__global__ __launch_bounds__(256) void affine_rand_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                          long total, long HW, uint64_t seed, double max_alpha,
                                                          int max_beta, int wrap) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / HW;
    const double alpha = crng_uniform(seed, n, 0) * max_alpha;
    const double beta = (double)(crng_below(seed, n, 1, (uint32_t)(2 * max_beta + 1)) - max_beta);
    const double v = (double)in[i] * alpha + beta;
    if (wrap) {
      long t = (long)trunc(v) % 256;
      out[i] = (uint8_t)(t < 0 ? t + 256 : t);
    } else {
      out[i] = sat_rint(v);
    }
  }
}

// ------------------------------------------------------------------ separable filters (P5/P6)
// Box / Gaussian: rows then columns with REFLECT_101, double accumulation in LDS.
// Taps at offsets -k/2 .. k-1-k/2 (even box sizes too, as the reference's cv2.blur).
__global__ __launch_bounds__(IMG_THREADS) void sep_filter_kernel(const uint8_t* __restrict__ in,
                                                                 uint8_t* __restrict__ out, int H, int W,
                                                                 const double* __restrict__ taps, int k) {
  extern __shared__ double s_tmp[];                      // [H*W] row-filtered
  __shared__ double s_k[32];
  const long base = (long)blockIdx.x * H * W;
  const int HW = H * W, r = k / 2;
  if (threadIdx.x < k) s_k[threadIdx.x] = taps[threadIdx.x];
  __syncthreads();
  for (int p = threadIdx.x; p < HW; p += IMG_THREADS) {
    const int y = p / W, x = p - y * W;
    double acc = 0.0;
    for (int i = 0; i < k; ++i) acc += s_k[i] * (double)in[base + (long)y * W + reflect101(x + i - r, W)];
    s_tmp[p] = acc;
  }
  __syncthreads();
  for (int p = threadIdx.x; p < HW; p += IMG_THREADS) {
    const int y = p / W, x = p - y * W;
    double acc = 0.0;
    for (int i = 0; i < k; ++i) acc += s_k[i] * s_tmp[reflect101(y + i - r, H) * W + x];
    out[base + p] = sat_rint(acc);
  }
}

// ------------------------------------------------------------------ rank filters (P7, P12, P13)
// op 0: median (REPLICATE border), 1: erode (min over in-bounds), 2: dilate (max).
__global__ __launch_bounds__(IMG_THREADS) void rank_filter_kernel(const uint8_t* __restrict__ in,
                                                                  uint8_t* __restrict__ out, int H, int W,
                                                                  int k, int op) {
  extern __shared__ uint8_t s_img[];
  const long base = (long)blockIdx.x * H * W;
  const int HW = H * W, r = k / 2;
  for (int p = threadIdx.x; p < HW; p += IMG_THREADS) s_img[p] = in[base + p];
  __syncthreads();
  for (int p = threadIdx.x; p < HW; p += IMG_THREADS) {
    const int y = p / W, x = p - y * W;
    if (op == 0) {
      // median of k*k (k <= 7): histogram-free rank selection over a register window
      uint8_t v[49];
      int n = 0;
      for (int dy = -r; dy <= r; ++dy)
        for (int dx = -r; dx <= r; ++dx) v[n++] = s_img[clampi(y + dy, H) * W + clampi(x + dx, W)];
      const int m = n / 2;
      int med = 0;
      for (int i = 0; i < n; ++i) {
        int lt = 0, le = 0;
        for (int j = 0; j < n; ++j) { lt += v[j] < v[i]; le += v[j] <= v[i]; }
        if (lt <= m && m < le) { med = v[i]; break; }
      }
      out[base + p] = (uint8_t)med;
    } else {
      int acc = op == 1 ? 255 : 0;
      for (int dy = -r; dy < k - r; ++dy) {            // k x k window at offset -k/2 (even k too)
        const int yy = y + dy;
        if (yy < 0 || yy >= H) continue;
        for (int dx = -r; dx < k - r; ++dx) {
          const int xx = x + dx;
          if (xx < 0 || xx >= W) continue;
          const int s = s_img[yy * W + xx];
          acc = op == 1 ? min(acc, s) : max(acc, s);
        }
      }
      out[base + p] = (uint8_t)acc;
    }
  }
}

// ------------------------------------------------------------------ histogram equalisation (P10)
__global__ __launch_bounds__(IMG_THREADS) void equalize_kernel(const uint8_t* __restrict__ in,
                                                               uint8_t* __restrict__ out, int HW) {
  __shared__ unsigned s_hist[256];
  __shared__ uint8_t s_lut[256];
  __shared__ int s_copy;
  const long base = (long)blockIdx.x * HW;
  s_hist[threadIdx.x] = 0;
  __syncthreads();
  for (int p = threadIdx.x; p < HW; p += IMG_THREADS) atomicAdd(&s_hist[in[base + p]], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {
    int first = -1, nz = 0;
    for (int b = 0; b < 256; ++b)
      if (s_hist[b]) { nz++; if (first < 0) first = b; }
    s_copy = (nz <= 1);
    if (!s_copy) {
      const unsigned cmin = s_hist[first];
      const double scale = 255.0 / (double)(HW - (int)cmin);
      unsigned cdf = 0;
      for (int b = 0; b < 256; ++b) {
        cdf += s_hist[b];
        double v = rint(((double)cdf - (double)cmin) * scale);
        v = v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v);
        s_lut[b] = b < first ? 0 : (uint8_t)v;
      }
    }
  }
  __syncthreads();
  for (int p = threadIdx.x; p < HW; p += IMG_THREADS) {
    const uint8_t v = in[base + p];
    out[base + p] = s_copy ? v : s_lut[v];
  }
}

// ------------------------------------------------------------------ CLAHE (P11)
// tiles x tiles grid (<= 8x8); tile histograms of the REFLECT_101-padded image in LDS,
// clip + uniform redistribution + residual stride, cdf LUTs, bilinear blend per pixel.
constexpr int CLAHE_MAX_TILES = 8;
__global__ __launch_bounds__(IMG_THREADS) void clahe_kernel(const uint8_t* __restrict__ in,
                                                            uint8_t* __restrict__ out, int H, int W,
                                                            int tiles, int clip) {
  extern __shared__ unsigned s_h[];                      // [tiles*tiles][256] hist, then LUT
  const long base = (long)blockIdx.x * H * W;
  const int th = (H + tiles - 1) / tiles, tw = (W + tiles - 1) / tiles;
  const int PH = th * tiles, PW = tw * tiles, T = tiles * tiles;
  for (int i = threadIdx.x; i < T * 256; i += IMG_THREADS) s_h[i] = 0;
  __syncthreads();
  for (int p = threadIdx.x; p < PH * PW; p += IMG_THREADS) {
    const int y = p / PW, x = p - y * PW;
    const uint8_t v = in[base + (long)reflect101(y, H) * W + reflect101(x, W)];
    atomicAdd(&s_h[((y / th) * tiles + x / tw) * 256 + v], 1u);
  }
  __syncthreads();
  const double lut_scale = 255.0 / (double)(th * tw);
  for (int t = threadIdx.x; t < T; t += IMG_THREADS) {
    unsigned* h = s_h + t * 256;
    if (clip > 0) {
      long excess = 0;
      for (int b = 0; b < 256; ++b)
        if ((int)h[b] > clip) { excess += (int)h[b] - clip; h[b] = clip; }
      const int add = (int)(excess / 256);
      int resid = (int)(excess % 256);
      for (int b = 0; b < 256; ++b) h[b] += add;
      if (resid) {
        const int step = max(256 / resid, 1);
        for (int b = 0; b < 256 && resid > 0; b += step) { h[b] += 1; --resid; }
      }
    }
    unsigned cdf = 0;
    for (int b = 0; b < 256; ++b) {
      cdf += h[b];
      double v = rint((double)cdf * lut_scale);
      h[b] = (unsigned)(v > 255.0 ? 255.0 : v);         // LUT in place
    }
  }
  __syncthreads();
  for (int p = threadIdx.x; p < H * W; p += IMG_THREADS) {
    const int y = p / W, x = p - y * W;
    const double ys = (y + 0.5) / th - 0.5, xs = (x + 0.5) / tw - 0.5;
    int y0 = (int)floor(ys), x0 = (int)floor(xs);
    const double fy = ys - y0, fx = xs - x0;
    int y1 = min(max(y0 + 1, 0), tiles - 1), x1 = min(max(x0 + 1, 0), tiles - 1);
    y0 = min(max(y0, 0), tiles - 1);
    x0 = min(max(x0, 0), tiles - 1);
    const int v = in[base + p];
    const double l00 = s_h[(y0 * tiles + x0) * 256 + v], l01 = s_h[(y0 * tiles + x1) * 256 + v];
    const double l10 = s_h[(y1 * tiles + x0) * 256 + v], l11 = s_h[(y1 * tiles + x1) * 256 + v];
    const double res = (l00 * (1 - fx) + l01 * fx) * (1 - fy) + (l10 * (1 - fx) + l11 * fx) * fy;
    out[base + p] = sat_rint(res);
  }
}

// Median with a compile-time window: the k*k values live in registers (a runtime-sized
// array went to scratch) and the rank selection is fully unrolled and branch-free.
template <int K>
__global__ __launch_bounds__(IMG_THREADS) void median_kernel(const uint8_t* __restrict__ in,
                                                             uint8_t* __restrict__ out, int H, int W) {
  extern __shared__ uint8_t s_img[];
  constexpr int R = K / 2, N = K * K, M = N / 2;
  const long base = (long)blockIdx.x * H * W;
  const int HW = H * W;
  for (int p = threadIdx.x; p < HW; p += IMG_THREADS) s_img[p] = in[base + p];
  __syncthreads();
  for (int p = threadIdx.x; p < HW; p += IMG_THREADS) {
    const int y = p / W, x = p - y * W;
    int v[N];
#pragma unroll
    for (int dy = 0; dy < K; ++dy)
#pragma unroll
      for (int dx = 0; dx < K; ++dx) v[dy * K + dx] = s_img[clampi(y + dy - R, H) * W + clampi(x + dx - R, W)];
    int med = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      int lt = 0, le = 0;
#pragma unroll
      for (int j = 0; j < N; ++j) { lt += v[j] < v[i]; le += v[j] <= v[i]; }
      med = (lt <= M && M < le) ? v[i] : med;
    }
    out[base + p] = (uint8_t)med;
  }
}

// ------------------------------------------------------------------ non-local means (P8)
// w(p,q) = exp(-max(0, d2)/h^2), d2 = mean squared 7x7 template difference (exact int
// sum), 21x21 search window, REFLECT_101 padding staged once in LDS.
__global__ __launch_bounds__(IMG_THREADS) void nlmeans_kernel(const uint8_t* __restrict__ in,
                                                              uint8_t* __restrict__ out, int H, int W,
                                                              double inv_h2, int tr, int sr) {
  extern __shared__ uint8_t s_p[];
  const int pad = tr + sr, PW = W + 2 * pad, PH = H + 2 * pad;
  const long base = (long)blockIdx.x * H * W;
  for (int p = threadIdx.x; p < PH * PW; p += IMG_THREADS) {
    const int y = p / PW, x = p - y * PW;
    s_p[p] = in[base + (long)reflect101(y - pad, H) * W + reflect101(x - pad, W)];
  }
  __syncthreads();
  const double inv_t2 = 1.0 / (double)((2 * tr + 1) * (2 * tr + 1));
  for (int p = threadIdx.x; p < H * W; p += IMG_THREADS) {
    const int y = p / W + pad, x = p - (p / W) * W + pad;
    double acc = 0.0, wsum = 0.0;
    for (int dy = -sr; dy <= sr; ++dy) {
      for (int dx = -sr; dx <= sr; ++dx) {
        int s = 0;
        for (int ty = -tr; ty <= tr; ++ty) {
          const uint8_t* a = s_p + (y + ty) * PW + x - tr;
          const uint8_t* b = s_p + (y + dy + ty) * PW + x + dx - tr;
          for (int tx = 0; tx <= 2 * tr; ++tx) {
            const int d = (int)a[tx] - (int)b[tx];
            s += d * d;
          }
        }
        const double w = exp(-(double)s * inv_t2 * inv_h2);
        acc += w * (double)s_p[(y + dy) * PW + x + dx];
        wsum += w;
      }
    }
    out[base + p] = sat_rint(acc / wsum);
  }
}

// Box-sum formulation (what the NumPy spec computes): for each of the 441 shifts the
// squared differences of the (H+2tr) x (W+2tr) template area are summed with a vertical
// then a horizontal running 7-window — ~13k integer ops per shift instead of 49 per
// pixel per shift — and every pixel's weight / accumulator update follows.  Sums are
// exact integers, the weight is the double exp of the spec.  LDS: padded image (uint8),
// the difference plane and the vertical sums (int).
__global__ __launch_bounds__(IMG_THREADS) void nlmeans_box_kernel(const uint8_t* __restrict__ in,
                                                                  uint8_t* __restrict__ out, int H, int W,
                                                                  double inv_h2, int tr, int sr) {
  extern __shared__ int s_nl[];
  const int pad = tr + sr, PW = W + 2 * pad, PH = H + 2 * pad;
  const int T = 2 * tr + 1, AW = W + 2 * tr, AH = H + 2 * tr;      // template area
  uint8_t* s_p = reinterpret_cast<uint8_t*>(s_nl);                  // [PH][PW]
  int* s_d = s_nl + (PH * PW + 3) / 4;                              // [AH][AW] squared diffs
  int* s_v = s_d + AH * AW;                                         // [H][AW] vertical sums
  const long base = (long)blockIdx.x * H * W;
  for (int p = threadIdx.x; p < PH * PW; p += IMG_THREADS) {
    const int y = p / PW, x = p - y * PW;
    s_p[p] = in[base + (long)reflect101(y - pad, H) * W + reflect101(x - pad, W)];
  }
  // every shift visits the same positions: their offsets are computed once (no integer
  // division inside the 441-shift loop)
  constexpr int MAXA = 8, MAXV = 8, MAXP = 4;  // area <= 2048, vertical <= 2048, pixels <= 1024
  int oa[MAXA], ov[MAXV], op_[MAXP], opp[MAXP];
#pragma unroll
  for (int q = 0; q < MAXA; ++q) {
    const int p = threadIdx.x + q * IMG_THREADS;
    const int y = p / AW, x = p - (p / AW) * AW;
    oa[q] = p < AH * AW ? (y + sr) * PW + x + sr : -1;            // area pixel in s_p
  }
#pragma unroll
  for (int q = 0; q < MAXV; ++q) {
    const int p = threadIdx.x + q * IMG_THREADS;
    ov[q] = p < H * AW ? p : -1;                                     // s_v index; s_d row y = p / AW
  }
#pragma unroll
  for (int q = 0; q < MAXP; ++q) {
    const int p = threadIdx.x + q * IMG_THREADS;
    const int y = p / W, x = p - (p / W) * W;
    op_[q] = p < H * W ? y * AW + x : -1;                            // s_v start of the window
    opp[q] = (y + pad) * PW + x + pad;                               // pixel in s_p
  }
  const float inv = (float)(inv_h2 / (double)(T * T));
  double acc[MAXP], wsum[MAXP];
#pragma unroll
  for (int q = 0; q < MAXP; ++q) acc[q] = wsum[q] = 0.0;
  __syncthreads();
  for (int dy = -sr; dy <= sr; ++dy) {
    for (int dx = -sr; dx <= sr; ++dx) {
      const int sh = dy * PW + dx;
      // 1) squared differences over the template area
#pragma unroll
      for (int q = 0; q < MAXA; ++q) {
        if (oa[q] < 0) break;
        const int d = (int)s_p[oa[q]] - (int)s_p[oa[q] + sh];
        s_d[threadIdx.x + q * IMG_THREADS] = d * d;
      }
      __syncthreads();
      // 2) vertical T-sums (s_d rows y..y+T-1 -> s_v[y]); same flat index p = y*AW + x
#pragma unroll
      for (int q = 0; q < MAXV; ++q) {
        if (ov[q] < 0) break;
        int sum = 0;
        for (int t = 0; t < T; ++t) sum += s_d[ov[q] + t * AW];
        s_v[ov[q]] = sum;
      }
      __syncthreads();
      // 3) horizontal T-sums -> weight -> this thread's pixels
#pragma unroll
      for (int q = 0; q < MAXP; ++q) {
        if (op_[q] < 0) break;
        int d2 = 0;
        for (int t = 0; t < T; ++t) d2 += s_v[op_[q] + t];
        const float w = __expf(-(float)d2 * inv);
        acc[q] += (double)(w * (float)s_p[opp[q] + sh]);
        wsum[q] += (double)w;
      }
      __syncthreads();                         // s_d / s_v are rewritten by the next shift
    }
  }
#pragma unroll
  for (int q = 0; q < MAXP; ++q) {
    const int p = threadIdx.x + q * IMG_THREADS;
    if (p < H * W) out[base + p] = sat_rint(acc[q] / wsum[q]);
  }
}

// ------------------------------------------------------------------ salt & pepper (P9)
// Coordinates are drawn on the host with the reference RNG order; per image: all salt
// (255) writes, barrier, then all pepper (0) writes.  Operates in place on ``img``.
__global__ __launch_bounds__(IMG_THREADS) void salt_pepper_kernel(uint8_t* __restrict__ img, int H, int W,
                                                                  const int* __restrict__ coords, int m) {
  const long base = (long)blockIdx.x * H * W;
  const int* c = coords + (long)blockIdx.x * 4 * m;      // [ys_salt, xs_salt, ys_pep, xs_pep]
  for (int i = threadIdx.x; i < m; i += IMG_THREADS) img[base + (long)c[i] * W + c[m + i]] = 255;
  __syncthreads();
  for (int i = threadIdx.x; i < m; i += IMG_THREADS) img[base + (long)c[2 * m + i] * W + c[3 * m + i]] = 0;
}

// counter-RNG variant: copies the image, then salt draw j = (y: 2+4j, x: 3+4j) and pepper
// draw j = (y: 4+4j, x: 5+4j) of image n (all salt, barrier, all pepper)
__global__ __launch_bounds__(IMG_THREADS) void salt_pepper_rand_kernel(const uint8_t* __restrict__ in,
                                                                       uint8_t* __restrict__ out, int H, int W,
                                                                       uint64_t seed, int m) {
  const long n = blockIdx.x, base = n * H * W;
  for (int p = threadIdx.x; p < H * W; p += IMG_THREADS) out[base + p] = in[base + p];
  __syncthreads();
  for (int j = threadIdx.x; j < m; j += IMG_THREADS)
    out[base + (long)crng_below(seed, n, 2 + 4 * (uint64_t)j, H) * W + crng_below(seed, n, 3 + 4 * (uint64_t)j, W)] = 255;
  __syncthreads();
  for (int j = threadIdx.x; j < m; j += IMG_THREADS)
    out[base + (long)crng_below(seed, n, 4 + 4 * (uint64_t)j, H) * W + crng_below(seed, n, 5 + 4 * (uint64_t)j, W)] = 0;
}

// ------------------------------------------------------------------ bicubic resize (P14)
// Separable 4-tap tables (index clamped = REPLICATE, a = -0.75) computed on the host.
__global__ __launch_bounds__(IMG_THREADS) void resize_kernel(const uint8_t* __restrict__ in,
                                                             uint8_t* __restrict__ out, int h, int w, int S,
                                                             const int* __restrict__ iy, const double* __restrict__ wy,
                                                             const int* __restrict__ ix, const double* __restrict__ wx) {
  extern __shared__ double s_rows[];                     // [S][w] row pass
  const long ib = (long)blockIdx.x * h * w, ob = (long)blockIdx.x * S * S;
  for (int p = threadIdx.x; p < S * w; p += IMG_THREADS) {
    const int oy = p / w, x = p - oy * w;
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc += (double)in[ib + (long)iy[oy * 4 + t] * w + x] * wy[oy * 4 + t];
    s_rows[p] = acc;
  }
  __syncthreads();
  for (int p = threadIdx.x; p < S * S; p += IMG_THREADS) {
    const int oy = p / S, ox = p - oy * S;
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc += s_rows[oy * w + ix[ox * 4 + t]] * wx[ox * 4 + t];
    out[ob + p] = sat_rint(acc);
  }
}

// ------------------------------------------------------------------ inference prep (C28)
// [N, 20, 20] grayscale (already bicubic-resized by the decoder) -> [N, 784]: centred in
// a 28x28 canvas at offset 4, > 150 -> 254 else 0 (construct_inference.py:312-330).
// float output: / 255 (the model input);  uint8 output: the 0 / 254 canvas itself, which
// the HIP forward kernels read like a dataset image (u8 / 255: the same float input).
template <class T>
__global__ __launch_bounds__(256) void infer_prep_kernel(const uint8_t* __restrict__ in, T* __restrict__ out,
                                                         long total) {
  constexpr float hi = sizeof(T) == 1 ? 254.f : 254.f / 255.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / 784;
    const int r = (int)(i - n * 784), y = r / 28 - 4, x = r % 28 - 4;
    float v = 0.f;
    if (y >= 0 && y < 20 && x >= 0 && x < 20) v = in[n * 400 + y * 20 + x] > 150 ? hi : 0.f;
    out[i] = (T)v;
  }
}

static unsigned grid_for(long total) {
  long g = (total + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

static bool big_lds(const void* fn) {
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) == hipSuccess;
}

}  // namespace csa

using namespace csa;

CSA_API int csa_img_flip(const uint8_t* in, uint8_t* out, int N, int H, int W, int mode, hipStream_t st) {
  if (N <= 0 || H <= 0 || W <= 0 || mode < 0 || mode > 2 || in == out) return -1;
  const long total = (long)N * H * W;
  hipLaunchKernelGGL(flip_kernel, dim3(grid_for(total)), dim3(256), 0, st, in, out, total, H, W, mode);
  return (int)hipGetLastError();
}

CSA_API int csa_img_affine(const uint8_t* in, uint8_t* out, int N, int H, int W, const double* alpha,
                           const double* beta, int wrap, hipStream_t st) {
  if (N <= 0 || H <= 0 || W <= 0) return -1;
  const long total = (long)N * H * W;
  hipLaunchKernelGGL(affine_kernel, dim3(grid_for(total)), dim3(256), 0, st, in, out, total, (long)H * W,
                     alpha, beta, wrap);
  return (int)hipGetLastError();
}

CSA_API int csa_img_affine_rand(const uint8_t* in, uint8_t* out, int N, int H, int W, unsigned long long seed,
                                double max_alpha, int max_beta, int wrap, hipStream_t st) {
  if (N <= 0 || H <= 0 || W <= 0 || max_beta < 0) return -1;
  const long total = (long)N * H * W;
  hipLaunchKernelGGL(affine_rand_kernel, dim3(grid_for(total)), dim3(256), 0, st, in, out, total, (long)H * W,
                     (uint64_t)seed, max_alpha, max_beta, wrap);
  return (int)hipGetLastError();
}

CSA_API int csa_img_salt_pepper_rand(const uint8_t* in, uint8_t* out, int N, int H, int W, unsigned long long seed,
                                     int m, hipStream_t st) {
  if (N <= 0 || m < 0 || in == out) return -1;
  hipLaunchKernelGGL(salt_pepper_rand_kernel, dim3(N), dim3(IMG_THREADS), 0, st, in, out, H, W, (uint64_t)seed, m);
  return (int)hipGetLastError();
}

CSA_API int csa_img_sep_filter(const uint8_t* in, uint8_t* out, int N, int H, int W, const double* taps, int k,
                               hipStream_t st) {
  if (N <= 0 || H * W > MAX_IMG_PIX / 2 || k < 1 || k > 31 || in == out) return -1;
  static bool attr = big_lds((const void*)sep_filter_kernel);
  (void)attr;
  hipLaunchKernelGGL(sep_filter_kernel, dim3(N), dim3(IMG_THREADS), sizeof(double) * H * W, st, in, out, H, W,
                     taps, k);
  return (int)hipGetLastError();
}

CSA_API int csa_img_rank_filter(const uint8_t* in, uint8_t* out, int N, int H, int W, int k, int op,
                                hipStream_t st) {
  if (N <= 0 || H * W > MAX_IMG_PIX || k < 1 || op < 0 || op > 2 || in == out) return -1;
  if (op == 0 && (k > 7 || (k & 1) == 0)) return -1;
  if (op == 0) {                         // median: register window, unrolled selection
    if (k == 1) hipLaunchKernelGGL(median_kernel<1>, dim3(N), dim3(IMG_THREADS), H * W, st, in, out, H, W);
    if (k == 3) hipLaunchKernelGGL(median_kernel<3>, dim3(N), dim3(IMG_THREADS), H * W, st, in, out, H, W);
    if (k == 5) hipLaunchKernelGGL(median_kernel<5>, dim3(N), dim3(IMG_THREADS), H * W, st, in, out, H, W);
    if (k == 7) hipLaunchKernelGGL(median_kernel<7>, dim3(N), dim3(IMG_THREADS), H * W, st, in, out, H, W);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(rank_filter_kernel, dim3(N), dim3(IMG_THREADS), H * W, st, in, out, H, W, k, op);
  return (int)hipGetLastError();
}

CSA_API int csa_img_equalize(const uint8_t* in, uint8_t* out, int N, int H, int W, hipStream_t st) {
  if (N <= 0 || H <= 0 || W <= 0) return -1;
  hipLaunchKernelGGL(equalize_kernel, dim3(N), dim3(IMG_THREADS), 0, st, in, out, H * W);
  return (int)hipGetLastError();
}

CSA_API int csa_img_clahe(const uint8_t* in, uint8_t* out, int N, int H, int W, int tiles, float clip_limit,
                          hipStream_t st) {
  if (N <= 0 || tiles < 1 || tiles > CLAHE_MAX_TILES || H < tiles || W < tiles || in == out) return -1;
  const int th = (H + tiles - 1) / tiles, tw = (W + tiles - 1) / tiles;
  const int c0 = (int)((double)clip_limit * th * tw / 256.0);
  const int clip = clip_limit > 0.f ? (c0 > 1 ? c0 : 1) : 0;
  static bool attr = big_lds((const void*)clahe_kernel);
  (void)attr;
  hipLaunchKernelGGL(clahe_kernel, dim3(N), dim3(IMG_THREADS), sizeof(unsigned) * tiles * tiles * 256, st, in, out,
                     H, W, tiles, clip);
  return (int)hipGetLastError();
}

CSA_API int csa_img_nlmeans(const uint8_t* in, uint8_t* out, int N, int H, int W, float h, int template_size,
                            int search_size, hipStream_t st) {
  const int tr = template_size / 2, sr = search_size / 2;
  if (N <= 0 || h <= 0.f || (H + 2 * (tr + sr)) * (W + 2 * (tr + sr)) > MAX_IMG_PIX || in == out) return -1;
  const int pad = tr + sr;
  if (H * W <= 4 * IMG_THREADS && (H + 2 * tr) * (W + 2 * tr) <= 8 * IMG_THREADS &&
      H * (W + 2 * tr) <= 8 * IMG_THREADS) {     // box-sum kernel's per-thread position tables
    const int AW = W + 2 * tr, AH = H + 2 * tr;
    const size_t lds = ((size_t)((H + 2 * pad) * (W + 2 * pad) + 3) / 4 + (size_t)AH * AW + (size_t)H * AW) * 4;
    if (lds <= 64 * 1024) {
      hipLaunchKernelGGL(nlmeans_box_kernel, dim3(N), dim3(IMG_THREADS), lds, st, in, out, H, W,
                         1.0 / ((double)h * (double)h), tr, sr);
      return (int)hipGetLastError();
    }
  }
  hipLaunchKernelGGL(nlmeans_kernel, dim3(N), dim3(IMG_THREADS), (H + 2 * pad) * (W + 2 * pad), st, in, out, H, W,
                     1.0 / ((double)h * (double)h), tr, sr);
  return (int)hipGetLastError();
}

CSA_API int csa_img_salt_pepper(uint8_t* img, int N, int H, int W, const int* coords, int m, hipStream_t st) {
  if (N <= 0 || m < 0) return -1;
  if (m == 0) return 0;
  hipLaunchKernelGGL(salt_pepper_kernel, dim3(N), dim3(IMG_THREADS), 0, st, img, H, W, coords, m);
  return (int)hipGetLastError();
}

CSA_API int csa_img_resize(const uint8_t* in, uint8_t* out, int N, int h, int w, int S, const int* iy,
                           const double* wy, const int* ix, const double* wx, hipStream_t st) {
  if (N <= 0 || S <= 0 || (long)S * w * 8 > 150 * 1024) return -1;
  static bool attr = big_lds((const void*)resize_kernel);
  (void)attr;
  hipLaunchKernelGGL(resize_kernel, dim3(N), dim3(IMG_THREADS), sizeof(double) * S * w, st, in, out, h, w, S, iy, wy,
                     ix, wx);
  return (int)hipGetLastError();
}

CSA_API int csa_img_infer_prep(const uint8_t* in, float* out, int N, hipStream_t st) {
  if (N <= 0) return -1;
  const long total = (long)N * 784;
  hipLaunchKernelGGL(infer_prep_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, in, out, total);
  return (int)hipGetLastError();
}

CSA_API int csa_img_infer_prep_u8(const uint8_t* in, uint8_t* out, int N, hipStream_t st) {
  if (N <= 0) return -1;
  const long total = (long)N * 784;
  hipLaunchKernelGGL(infer_prep_kernel<uint8_t>, dim3(grid_for(total)), dim3(256), 0, st, in, out, total);
  return (int)hipGetLastError();
}
