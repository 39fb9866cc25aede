// C ABI of libhybridflux (include/hybridflux.h): model handles, weight
// packing into MFMA fragment order, argument validation, launch sequencing.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "hf_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}
int fail_hip(hipError_t e, const char *what) {
  return fail(HF_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HF_CHECK_HIP(expr, what)                  \
  do {                                            \
    hipError_t _e = (expr);                       \
    if (_e != hipSuccess) return fail_hip(_e, what); \
  } while (0)

}  // namespace

struct hf_model {
  int in_dim = 0, hidden = 0, layers = 0, wdtype = 0;
  bool chain_ok = false;  // fused chain kernels need in_dim 4, hidden 128, f32
  float *dev = nullptr;   // single device allocation holding every buffer
  hf::ChainW chain{};
  hf::GraphW graph{};
};

namespace {

// Offsets of each parameter inside the reference-ordered flat array.
struct Layout {
  int64_t w_in, b_in, w_l, b_l, w_e, b_e, w_2, b_2, total;
  Layout(int in, int H, int L) {
    int64_t o = 0;
    w_in = o; o += (int64_t)H * in;
    b_in = o; o += H;
    w_l = o;  // per layer: weight [H][2H] then bias [H]
    b_l = -1;
    o += (int64_t)L * ((int64_t)H * 2 * H + H);
    w_e = o; o += (int64_t)H * 2 * H;
    b_e = o; o += H;
    w_2 = o; o += H;
    b_2 = o; o += 1;
    total = o;
  }
};

// Pack the reference weights into the A-fragment order of chain_gnn.hip.
//  k-step s of a 128-wide half, lane l: k = 16*(s>>2) + 4*(l>>4) + (s&3),
//  output row n = 16*nt + (l&15).
int kperm(int s, int lane) { return 16 * (s >> 2) + 4 * (lane >> 4) + (s & 3); }

// Chain-kernel packing (chain_f32.hip / chain_k32.hip; layouts in hf_internal.h).
//  f32 `stream`: chain_chunks chunks of [j 8][lane 64][4] floats.  Update-layer
//    chunk (l, gi): k-step s = 4gi + (j>>1), output tile nt = 4(j&1) + c,
//    k = (s < 32 ? 0 : 128) + kperm(s % 32, lane).  Readout chunk (ot, hh):
//    k-step s = 16hh + 2j + (c>>1), c&1 selects P = W_e[:, :H] or Q = W_e[:, H:].
//  k32 `stream` (f16x3, bf16): per layer units (pair q = 0..3, kb = 0..3) of
//    [i = 2t + (W_a|W_b)][term][lane][e 0..7] 16-bit values with output tile
//    nt = 2q + t and k = (W_b ? 128 : 0) + 16(2kb + (e>>2)) + 4(lane>>4) + (e&3);
//    then per readout tile ot one chunk [j = 2kb + (P|Q)][term][lane][e].
//    f16x3: term 0 = fp16(w), term 1 = fp16(w - term0); bf16: one bf16(w) term.
//  Row n = 16*tile + (lane&15) throughout.
//  small (f32): win [j 2][lane][4] (tile nt = 4j + c, column k = lane>>4), then
//    b_in, b_l[L], b_e, w2; b2 as a scalar.  In bf16 mode every weight matrix
//    (incl. W_in, w2) is rounded to bf16 values; biases stay f32.
uint16_t to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
uint16_t f16_bits(_Float16 h) {
  uint16_t b;
  std::memcpy(&b, &h, 2);
  return b;
}

struct ChainPack {
  std::vector<unsigned char> stream;
  std::vector<float> small;
  int64_t o_win = 0, o_bin = 0, o_bl = 0, o_be = 0, o_w2 = 0;
  float b2 = 0.f;
};

template <class T>
void put(std::vector<unsigned char> &out, T v) {
  const unsigned char *b = reinterpret_cast<const unsigned char *>(&v);
  out.insert(out.end(), b, b + sizeof(T));
}

void pack_chain(const float *p, int L, int prec, ChainPack &P) {
  using hf::kH;
  using hf::kKS;
  using hf::kNT;
  const Layout lay(hf::kIn, kH, L);
  auto layer_w = [&](int l) { return p + lay.w_l + (int64_t)l * ((int64_t)kH * 2 * kH + kH); };
  auto q = [&](float v) { return prec == hf::kPrecBF16 ? bf16_to_f32(to_bf16(v)) : v; };
  std::vector<unsigned char> &out = P.stream;
  out.clear();
  if (prec == hf::kPrecF32) {
    for (int c = 0; c < hf::chain_chunks(L, prec); ++c)
      for (int j = 0; j < 8; ++j)
        for (int lane = 0; lane < 64; ++lane)
          for (int cc = 0; cc < 4; ++cc) {
            float v;
            if (c < 16 * L) {
              const int l = c / 16, gi = c % 16;
              const int s = 4 * gi + (j >> 1), nt = 4 * (j & 1) + cc;
              const int k = (s < kKS ? 0 : kH) + kperm(s % kKS, lane);
              v = layer_w(l)[(int64_t)(16 * nt + (lane & 15)) * 2 * kH + k];
              // the 1/deg = 1/2 of the mean aggregation is folded into W_b (an exact
              // power-of-two scaling: w*(s/2) == (w/2)*s bit for bit)
              if (s >= kKS) v *= 0.5f;
            } else {
              const int r = c - 16 * L, ot = r / 2, hh = r % 2;
              const int s = 16 * hh + 2 * j + (cc >> 1), pq = cc & 1;
              v = p[lay.w_e + (int64_t)(16 * ot + (lane & 15)) * 2 * kH + pq * kH + kperm(s, lane)];
            }
            put(out, v);
          }
  } else {
    const int terms = prec == hf::kPrecF16x3 ? 2 : 1;
    // one 16-byte fragment (8 values) of row `row`, k-block kb, column offset kbase
    auto frag = [&](const float *W, int64_t ld, int row, int kbase, int kb, int lane, int term, bool halve_b) {
      for (int e = 0; e < 8; ++e) {
        const int k = kbase + 16 * (2 * kb + (e >> 2)) + 4 * (lane >> 4) + (e & 3);
        // bf16: the 1/deg = 1/2 of the mean aggregation is folded into W_b
        // (chain_bf16.hip, input-side aggregation); exact, bf16(w/2) == bf16(w)/2
        const float w = W[(int64_t)row * ld + k] * (halve_b && kbase == kH ? 0.5f : 1.0f);
        if (prec == hf::kPrecBF16) {
          put(out, to_bf16(w));
        } else {
          const _Float16 hi = (_Float16)w;
          const _Float16 lo = (_Float16)(w - (float)hi);
          put(out, f16_bits(term == 0 ? hi : lo));
        }
      }
    };
    // chain_bf16.hip and chain_k32.hip walk a layer by output pair q (tiles
    // 2q, 2q+1), k-block kb within it: unit (q, kb) = fragments i = 2t +
    // (W_a | W_b) of tile 2q + t, each [term][lane][e].  bf16 folds the 1/deg
    // into W_b (input-side aggregation); f16x3 applies it to G in the epilogue.
    for (int l = 0; l < L; ++l)
      for (int qp = 0; qp < 4; ++qp)
        for (int kb = 0; kb < 4; ++kb)
          for (int i = 0; i < 4; ++i)
            for (int t = 0; t < terms; ++t)
              for (int lane = 0; lane < 64; ++lane) {
                const int nt = 2 * qp + (i >> 1), ab = i & 1;
                frag(layer_w(l), 2 * kH, 16 * nt + (lane & 15), ab * kH, kb, lane, t, prec == hf::kPrecBF16);
              }
    for (int ot = 0; ot < kNT; ++ot)
      for (int j = 0; j < 8; ++j)
        for (int t = 0; t < terms; ++t)
          for (int lane = 0; lane < 64; ++lane) {
            const int kb = j >> 1, pq = j & 1;
            frag(p + lay.w_e, 2 * kH, 16 * ot + (lane & 15), pq * kH, kb, lane, t, false);
          }
    // bf16: a copy of the first two units (8 KiB) after the pass, so the
    // super-window flux kernel can read the pass as 16 KiB chunks offset by two
    // units (hf::kBF16StreamTail; chain_bf16.hip CoreBF16<..., XCH>)
    if (prec == hf::kPrecBF16) {
      const std::vector<unsigned char> head(out.begin(), out.begin() + hf::kBF16StreamTail);
      out.insert(out.end(), head.begin(), head.end());
    }
  }
  std::vector<float> &sm = P.small;
  sm.clear();
  P.o_win = 0;
  for (int j = 0; j < 2; ++j)
    for (int lane = 0; lane < 64; ++lane)
      for (int cc = 0; cc < 4; ++cc) {
        const int nt = 4 * j + cc;
        sm.push_back(q(p[lay.w_in + (int64_t)(16 * nt + (lane & 15)) * hf::kIn + (lane >> 4)]));
      }
  P.o_bin = (int64_t)sm.size();
  sm.insert(sm.end(), p + lay.b_in, p + lay.b_in + kH);
  P.o_bl = (int64_t)sm.size();
  for (int l = 0; l < L; ++l) sm.insert(sm.end(), layer_w(l) + (int64_t)kH * 2 * kH, layer_w(l) + (int64_t)kH * 2 * kH + kH);
  P.o_be = (int64_t)sm.size();
  sm.insert(sm.end(), p + lay.b_e, p + lay.b_e + kH);
  P.o_w2 = (int64_t)sm.size();
  for (int i = 0; i < kH; ++i) sm.push_back(q(p[lay.w_2 + i]));
  P.b2 = p[lay.b_2];
}

hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

bool fused_nx(int nx) { return nx == 16 || nx == 32 || nx == 48 || nx == 64; }

int check_device() {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return fail(HF_EHIP, "no HIP device visible: libhybridflux has no CPU path");
  return HF_OK;
}

int chain_usable(const hf_model *m) {
  if (!m->chain_ok)
    return fail(HF_EUNSUPPORTED,
                "chain kernels are specialised to FluxGNN(input_dim=4, hidden_dim=128, num_layers<=8) float32 "
                "(src/config.py:19-23); use hf_graph_flux for other widths");
  return HF_OK;
}

}  // namespace

extern "C" {

#ifndef HF_SOURCE_HASH
#define HF_SOURCE_HASH "unknown"
#endif
#ifndef HF_BUILD_FLAGS
#define HF_BUILD_FLAGS ""
#endif
// "hybridflux <version> gfx950 src:<hash>": the hash covers every source,
// header and the Makefile the library was built from, and the extra compiler
// flags (Makefile SRC_HASH).  A build with extra flags (HF_DIAG_* timing
// diagnostics, HF_EXP_* experiments) says so: "... src:<hash> flags:<flags>".
const char *hf_version(void) {
  return sizeof(HF_BUILD_FLAGS) > 1 ? "hybridflux 0.2 gfx950 src:" HF_SOURCE_HASH " flags:" HF_BUILD_FLAGS
                                    : "hybridflux 0.2 gfx950 src:" HF_SOURCE_HASH;
}

const char *hf_last_error(void) { return g_err.c_str(); }

int hf_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int64_t hf_model_param_count(int in_dim, int hidden, int layers) {
  if (in_dim <= 0 || hidden <= 0 || layers < 0) return -1;
  return Layout(in_dim, hidden, layers).total;
}

int hf_model_create(const float *host_params, int in_dim, int hidden, int layers, int wdtype,
                    hf_model_t *out) {
  if (!out) return fail(HF_EINVAL, "hf_model_create: out is NULL");
  *out = nullptr;
  if (!host_params) return fail(HF_EINVAL, "hf_model_create: host_params is NULL");
  if (in_dim <= 0 || hidden <= 0 || layers < 0)
    return fail(HF_EINVAL, "hf_model_create: dimensions must be positive");
  if (wdtype != HF_WDTYPE_F32 && wdtype != HF_WDTYPE_BF16 && wdtype != HF_WDTYPE_F16X3)
    return fail(HF_EINVAL, "hf_model_create: unknown wdtype");
  if (int rc = check_device()) return rc;

  const Layout lay(in_dim, hidden, layers);
  hf_model *m = new hf_model();
  m->in_dim = in_dim;
  m->hidden = hidden;
  m->layers = layers;
  m->wdtype = wdtype;
  m->chain_ok = (in_dim == hf::kIn && hidden == hf::kH && layers <= hf::kMaxChainLayers);

  // natural copy (graph path) followed by the packed copy (chain path)
  ChainPack pk;
  if (m->chain_ok) pack_chain(host_params, layers, wdtype, pk);
  // natural layer weights are split into contiguous [L][H][2H] and [L][H]
  std::vector<float> nat((size_t)lay.total);
  {
    int64_t o = 0;
    auto put = [&](int64_t src, int64_t n) {
      std::memcpy(nat.data() + o, host_params + src, sizeof(float) * n);
      o += n;
    };
    put(lay.w_in, (int64_t)hidden * in_dim);
    put(lay.b_in, hidden);
    for (int l = 0; l < layers; ++l)
      put(lay.w_l + (int64_t)l * ((int64_t)hidden * 2 * hidden + hidden), (int64_t)hidden * 2 * hidden);
    for (int l = 0; l < layers; ++l)
      put(lay.w_l + (int64_t)l * ((int64_t)hidden * 2 * hidden + hidden) + (int64_t)hidden * 2 * hidden,
          hidden);
    put(lay.w_e, (int64_t)hidden * 2 * hidden);
    put(lay.b_e, hidden);
    put(lay.w_2, hidden);
    put(lay.b_2, 1);
  }
  const size_t nat_bytes = (sizeof(float) * nat.size() + 255) & ~size_t(255);
  const size_t stream_bytes = (pk.stream.size() + 255) & ~size_t(255);
  const size_t small_bytes = (sizeof(float) * pk.small.size() + 255) & ~size_t(255);
  const size_t bytes = nat_bytes + stream_bytes + small_bytes;
  hipError_t e = hipMalloc(&m->dev, bytes);
  if (e != hipSuccess) {
    delete m;
    return fail(HF_ENOMEM, std::string("hf_model_create: hipMalloc: ") + hipGetErrorString(e));
  }
  char *base = reinterpret_cast<char *>(m->dev);
  e = hipMemcpy(base, nat.data(), sizeof(float) * nat.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && !pk.stream.empty())
    e = hipMemcpy(base + nat_bytes, pk.stream.data(), pk.stream.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && !pk.small.empty())
    e = hipMemcpy(base + nat_bytes + stream_bytes, pk.small.data(), sizeof(float) * pk.small.size(),
                  hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(m->dev);
    delete m;
    return fail_hip(e, "hf_model_create: upload");
  }
  {
    const float *d = m->dev;
    int64_t o = 0;
    hf::GraphW &g = m->graph;
    g.in_dim = in_dim;
    g.hidden = hidden;
    g.layers = layers;
    g.w_in = d + o; o += (int64_t)hidden * in_dim;
    g.b_in = d + o; o += hidden;
    g.w_l = d + o; o += (int64_t)layers * hidden * 2 * hidden;
    g.b_l = d + o; o += (int64_t)layers * hidden;
    g.lsw = (int64_t)hidden * 2 * hidden;
    g.lsb = hidden;
    g.w_e = d + o; o += (int64_t)hidden * 2 * hidden;
    g.b_e = d + o; o += hidden;
    g.w_2 = d + o; o += hidden;
    g.b_2 = d + o;
  }
  if (m->chain_ok) {
    const float *d = reinterpret_cast<const float *>(base + nat_bytes + stream_bytes);
    hf::ChainW &c = m->chain;
    c.stream = base + nat_bytes;
    c.prec = wdtype;
    c.win = d + pk.o_win;
    c.bin = d + pk.o_bin;
    c.bl = d + pk.o_bl;
    c.be = d + pk.o_be;
    c.w2 = d + pk.o_w2;
    c.b2 = pk.b2;
    c.layers = layers;
  }
  *out = m;
  return HF_OK;
}

void hf_model_destroy(hf_model_t model) {
  if (!model) return;
  if (model->dev) (void)hipFree(model->dev);
  delete model;
}

int hf_chain_flux(hf_model_t m, const float *nf, int B, int nx, float *fe, float *ff, void *stream) {
  if (!m) return fail(HF_EINVAL, "hf_chain_flux: NULL model");
  if (B < 0 || nx < 1) return fail(HF_EINVAL, "hf_chain_flux: need B >= 0 and nx >= 1");
  if (B == 0) return HF_OK;
  if (!nf) return fail(HF_EINVAL, "hf_chain_flux: NULL node features");
  if (int rc = chain_usable(m)) return rc;
  if (!fe && !ff) return HF_OK;
  HF_CHECK_HIP(hf::launch_chain_flux(m->chain, nf, nullptr, 0, nullptr, B, nx, fe, ff, as_stream(stream)),
               "hf_chain_flux");
  return HF_OK;
}

int64_t hf_graph_workspace_bytes(hf_model_t m, int64_t N, int64_t E) {
  if (!m || N < 0 || E < 0) return -1;
  return hf::graph_workspace_bytes(m->graph, N, E);
}

int hf_graph_flux(hf_model_t m, const float *nf, int64_t N, const int64_t *ei, int64_t E,
                  float *flux, void *ws, void *stream) {
  if (!m) return fail(HF_EINVAL, "hf_graph_flux: NULL model");
  if (N < 0 || E < 0) return fail(HF_EINVAL, "hf_graph_flux: negative size");
  if (E == 0) return HF_OK;
  if (N == 0) return fail(HF_EINVAL, "hf_graph_flux: edges without nodes");
  if (!nf || !ei || !flux || !ws) return fail(HF_EINVAL, "hf_graph_flux: NULL pointer");
  if (N > 0x7fffffffLL || E > 0x7fffffffLL) return fail(HF_EUNSUPPORTED, "hf_graph_flux: > 2^31 nodes/edges");
  HF_CHECK_HIP(hf::launch_graph_flux(m->graph, nf, N, ei, E, flux, ws, as_stream(stream)), "hf_graph_flux");
  return HF_OK;
}

// ------------------------------------------------------------------ training
static int train_dims_ok(int in_dim, int hidden, int layers) {
  return in_dim >= 1 && hidden >= 1 && layers >= 0 && layers <= hf::kMaxChainLayers;
}

int64_t hf_graph_tape_bytes(int in_dim, int hidden, int layers, int64_t N, int64_t E) {
  if (!train_dims_ok(in_dim, hidden, layers) || N < 0 || E < 0) return -1;
  return hf::graph_tape_bytes(hf::graph_view_state_dict(nullptr, in_dim, hidden, layers), N, E);
}

int64_t hf_graph_backward_workspace_bytes(int in_dim, int hidden, int layers, int64_t N, int64_t E) {
  if (!train_dims_ok(in_dim, hidden, layers) || N < 0 || E < 0) return -1;
  return hf::graph_backward_ws_bytes(hf::graph_view_state_dict(nullptr, in_dim, hidden, layers), N, E);
}

static int train_args(const char *fn, int in_dim, int hidden, int layers, int64_t N, int64_t E) {
  if (!train_dims_ok(in_dim, hidden, layers))
    return fail(HF_EINVAL, std::string(fn) + ": bad model dimensions (layers <= 8)");
  if (N < 0 || E < 0) return fail(HF_EINVAL, std::string(fn) + ": negative size");
  if (E > 0 && N == 0) return fail(HF_EINVAL, std::string(fn) + ": edges without nodes");
  if (N > 0x7fffffffLL || E > 0x7fffffffLL) return fail(HF_EUNSUPPORTED, std::string(fn) + ": > 2^31 nodes/edges");
  return HF_OK;
}

static int chain_args(const char *fn, int chain_nx, int64_t N, int64_t E) {
  if (chain_nx < 0 || (chain_nx > 0 && (N % chain_nx != 0 || E != 2 * N)))
    return fail(HF_EINVAL, std::string(fn) + ": chain_nx must divide N with E == 2N (or be 0)");
  return HF_OK;
}

int hf_graph_forward_train(const float *params, int in_dim, int hidden, int layers, const float *nf, int64_t N,
                           const int64_t *ei, int64_t E, int chain_nx, float *flux, void *tape, void *stream) {
  if (int rc = train_args("hf_graph_forward_train", in_dim, hidden, layers, N, E)) return rc;
  if (int rc = chain_args("hf_graph_forward_train", chain_nx, N, E)) return rc;
  if (E == 0) return HF_OK;
  if (!params || !nf || !ei || !flux || !tape) return fail(HF_EINVAL, "hf_graph_forward_train: NULL pointer");
  const hf::GraphW w = hf::graph_view_state_dict(params, in_dim, hidden, layers);
  HF_CHECK_HIP(hf::launch_graph_forward_train(w, nf, N, ei, E, chain_nx, flux, tape, as_stream(stream)),
               "hf_graph_forward_train");
  return HF_OK;
}

int hf_graph_backward(const float *params, int in_dim, int hidden, int layers, const float *nf, int64_t N,
                      const int64_t *ei, int64_t E, int chain_nx, const void *tape, const float *grad_flux,
                      float *grad_params, float *grad_nf, void *ws, void *stream) {
  if (int rc = train_args("hf_graph_backward", in_dim, hidden, layers, N, E)) return rc;
  if (int rc = chain_args("hf_graph_backward", chain_nx, N, E)) return rc;
  if (!params || !grad_params) return fail(HF_EINVAL, "hf_graph_backward: NULL pointer");
  if (E > 0 && (!nf || !ei || !tape || !grad_flux || !ws)) return fail(HF_EINVAL, "hf_graph_backward: NULL pointer");
  const hf::GraphW w = hf::graph_view_state_dict(params, in_dim, hidden, layers);
  HF_CHECK_HIP(hf::launch_graph_backward(w, nf, N, ei, E, chain_nx, tape, grad_flux, grad_params, grad_nf, ws,
                                         as_stream(stream)),
               "hf_graph_backward");
  return HF_OK;
}

int64_t hf_ablation_loss_workspace_bytes(int B, int nx) {
  if (B < 0 || nx < 1) return -1;
  return hf::ablation_loss_ws_bytes(B, nx);
}

int hf_ablation_loss_ex(const float *fe, const float *st, const float *ft, const float *sn, int B, int nx, float c,
                        float dx, const float *lam, int rollout_steps, float dt, const double *pc, float *loss,
                        float *flux_loss, float *dfe, void *ws, int64_t ws_bytes, void *stream) {
  if (B < 1 || nx < 1) return fail(HF_EINVAL, "hf_ablation_loss: need B >= 1, nx >= 1");
  if (!fe || !st || !ft || !sn || !lam || !pc || !loss || !flux_loss || !dfe || !ws)
    return fail(HF_EINVAL, "hf_ablation_loss: NULL pointer");
  if (ws_bytes < hf::ablation_loss_ws_bytes(B, nx))
    return fail(HF_EINVAL, "hf_ablation_loss: workspace smaller than hf_ablation_loss_workspace_bytes");
  if (rollout_steps < 0) return fail(HF_EINVAL, "hf_ablation_loss_ex: rollout_steps < 0");
  if (rollout_steps > hf::kLossMaxRollout && lam[4] > 0.f)
    return fail(HF_EUNSUPPORTED, "hf_ablation_loss_ex: rollout_steps > 3 needs model forwards on later states "
                                 "(pass lam[4] = 0 and add the term from those forwards)");
  HF_CHECK_HIP(hf::launch_ablation_loss(fe, st, ft, sn, B, nx, c, dx, lam, rollout_steps, dt, pc, loss, flux_loss, dfe,
                                        ws, as_stream(stream)),
               "hf_ablation_loss");
  return HF_OK;
}

int hf_ablation_loss(const float *fe, const float *st, const float *ft, const float *sn, int B, int nx, float c,
                     float dx, const float *lam, const double *pc, float *loss, float *flux_loss, float *dfe, void *ws,
                     int64_t ws_bytes, void *stream) {
  if (!lam) return fail(HF_EINVAL, "hf_ablation_loss: NULL pointer");
  const float lam5[5] = {lam[0], lam[1], lam[2], lam[3], 0.f};
  return hf_ablation_loss_ex(fe, st, ft, sn, B, nx, c, dx, lam5, 0, 0.f, pc, loss, flux_loss, dfe, ws, ws_bytes,
                             stream);
}

int hf_chain_batch_gather(const int64_t *idx, int B, const float *st_all, const float *ft_all, const float *sn_all,
                          int64_t N, int nx, const float *x, float *st, float *ft, float *sn, float *nf,
                          void *stream) {
  if (B < 0 || nx < 1 || N < 1) return fail(HF_EINVAL, "hf_chain_batch_gather: need B >= 0, nx >= 1, N >= 1");
  if (B > 0 && (!idx || !st_all || !ft_all || !sn_all || !x || !st || !ft || !sn || !nf))
    return fail(HF_EINVAL, "hf_chain_batch_gather: NULL pointer");
  HF_CHECK_HIP(hf::launch_chain_batch_gather(idx, B, st_all, ft_all, sn_all, N, nx, x, st, ft, sn, nf,
                                             as_stream(stream)),
               "hf_chain_batch_gather");
  return HF_OK;
}

int hf_adam_flat(float *params, const float *grads, float *exp_avg, float *exp_avg_sq, int64_t n, float *step,
                 unsigned *done, float lr, float beta1, float beta2, float eps, void *stream) {
  if (n < 0) return fail(HF_EINVAL, "hf_adam_flat: n < 0");
  if (n > 0 && (!params || !grads || !exp_avg || !exp_avg_sq || !step || !done))
    return fail(HF_EINVAL, "hf_adam_flat: NULL pointer");
  if (n == 0) return HF_OK;
  HF_CHECK_HIP(hf::launch_adam_flat(params, grads, exp_avg, exp_avg_sq, n, step, done, lr, beta1, beta2, eps,
                                    as_stream(stream)),
               "hf_adam_flat");
  return HF_OK;
}

// ------------------------------------------------------- PureGNN / PINN
int64_t hf_pure_gnn_param_count(int in_dim, int hidden, int layers) {
  if (in_dim < 1 || hidden < 1 || layers < 0) return -1;
  const int64_t H = hidden;
  return H * in_dim + H + layers * (2 * H * H + H) + H * H + H + 3 * H + 3;
}

int64_t hf_pure_gnn_workspace_bytes(int hidden, int64_t N, int64_t E) {
  if (hidden < 1 || N < 0 || E < 0) return -1;
  return hf::pure_gnn_ws_bytes(hidden, N, E);
}

int64_t hf_pure_gnn_run_workspace_bytes(int hidden, int B, int nx, int T) {
  if (hidden < 1 || B < 0 || nx < 1 || T < 0) return -1;
  return hf::pure_gnn_run_ws_bytes(hidden, B, nx, T);
}

int hf_pure_gnn_forward(const float *params, int in_dim, int hidden, int layers, const float *nf, int64_t N,
                        const int64_t *ei, int64_t E, int chain_nx, float *delta, void *ws, void *stream) {
  if (in_dim < 1 || hidden < 1 || layers < 0) return fail(HF_EINVAL, "hf_pure_gnn_forward: bad model dimensions");
  if (N < 0 || E < 0) return fail(HF_EINVAL, "hf_pure_gnn_forward: negative size");
  if (E > 0 && N == 0) return fail(HF_EINVAL, "hf_pure_gnn_forward: edges without nodes");
  if (int rc = chain_args("hf_pure_gnn_forward", chain_nx, N, E)) return rc;
  if (N == 0) return HF_OK;
  if (!params || !nf || !delta || !ws || (E > 0 && !ei)) return fail(HF_EINVAL, "hf_pure_gnn_forward: NULL pointer");
  HF_CHECK_HIP(hf::launch_pure_gnn_forward(params, in_dim, hidden, layers, nf, N, ei, E, chain_nx, delta, ws,
                                           as_stream(stream)),
               "hf_pure_gnn_forward");
  return HF_OK;
}

int hf_pure_gnn_run(const float *params, int hidden, int layers, const float *state0, float *final_state,
                    const float *x, int B, int nx, int T, float *traj, void *ws, void *stream) {
  if (hidden < 1 || layers < 0 || B < 0 || nx < 1 || T < 0) return fail(HF_EINVAL, "hf_pure_gnn_run: bad argument");
  if (B == 0) return HF_OK;
  if (!params || !state0 || !final_state || !x) return fail(HF_EINVAL, "hf_pure_gnn_run: NULL pointer");
  // the one-launch rollout runs on nn.Linear's rows without a workspace (its
  // packed copy is an optimisation); the per-step path needs its scratch
  if (!ws && !hf::pure_gnn_run_ws_optional(hidden, nx, T) && hf::pure_gnn_run_ws_bytes(hidden, B, nx, T) > 0)
    return fail(HF_EINVAL, "hf_pure_gnn_run: NULL workspace (hf_pure_gnn_run_workspace_bytes > 0 for this shape)");
  HF_CHECK_HIP(hf::launch_pure_gnn_run(params, hidden, layers, state0, final_state, x, B, nx, T, traj, ws,
                                       as_stream(stream)),
               "hf_pure_gnn_run");
  return HF_OK;
}

int64_t hf_pinn_param_count(int dim, int hidden, int layers) {
  if (dim < 1 || hidden < 1 || layers < 2 || layers > hf::kMaxChainLayers) return -1;
  const int64_t D = dim, H = hidden;
  return (D * H + H) + (layers - 2) * (H * H + H) + (H * D + D);
}

int64_t hf_pinn_workspace_bytes(int dim, int hidden, int64_t B) {
  if (dim < 1 || hidden < 1 || B < 0) return -1;
  return hf::pinn_run_ws_bytes(dim, hidden, B);
}

static int pinn_args(const char *fn, int dim, int hidden, int layers, int64_t B) {
  if (dim < 1 || hidden < 1 || layers < 2 || layers > hf::kMaxChainLayers || B < 0)
    return fail(HF_EINVAL, std::string(fn) + ": bad argument (2 <= layers <= 8)");
  return HF_OK;
}

int hf_pinn_forward(const float *params, int dim, int hidden, int layers, const float *state, float *out, int64_t B,
                    void *ws, void *stream) {
  if (int rc = pinn_args("hf_pinn_forward", dim, hidden, layers, B)) return rc;
  if (B == 0) return HF_OK;
  if (!params || !state || !out) return fail(HF_EINVAL, "hf_pinn_forward: NULL pointer");
  if (!ws && hf::pinn_run_ws_bytes(dim, hidden, B) > 0)
    return fail(HF_EINVAL, "hf_pinn_forward: NULL workspace (hf_pinn_workspace_bytes > 0 for this shape)");
  if (state == out) return fail(HF_EINVAL, "hf_pinn_forward: state and out must not alias");
  HF_CHECK_HIP(hf::launch_pinn_forward(params, dim, hidden, layers, state, out, B, ws, as_stream(stream)),
               "hf_pinn_forward");
  return HF_OK;
}

int hf_pinn_run(const float *params, int dim, int hidden, int layers, const float *state0, float *final_state,
                int64_t B, int T, float *traj, void *ws, void *stream) {
  if (int rc = pinn_args("hf_pinn_run", dim, hidden, layers, B)) return rc;
  if (T < 0) return fail(HF_EINVAL, "hf_pinn_run: T < 0");
  if (B == 0) return HF_OK;
  if (!params || !state0 || !final_state) return fail(HF_EINVAL, "hf_pinn_run: NULL pointer");
  if (!ws && T > 0 && hf::pinn_run_ws_bytes(dim, hidden, B) > 0)
    return fail(HF_EINVAL, "hf_pinn_run: NULL workspace (hf_pinn_workspace_bytes > 0 for this shape)");
  HF_CHECK_HIP(hf::launch_pinn_run(params, dim, hidden, layers, state0, final_state, B, T, traj, ws,
                                   as_stream(stream)),
               "hf_pinn_run");
  return HF_OK;
}

int hf_poisson_plan_len(int nx) { return nx < 1 ? -1 : hf::poisson_plan_len(nx); }

int hf_poisson_coeffs(int nx, double length, double *c) {
  if (nx < 1 || !(length > 0) || !c) return fail(HF_EINVAL, "hf_poisson_coeffs: bad argument");
  // E = Re(ifft(i fft(rho)/k)), k_q = 2 pi q'/L over the signed fftfreq q'
  // (src/baseline_solver.py:26).  Pairing +-q' gives
  //   c[d] = -(L / (pi nx)) * sum_{q'=1}^{ceil(nx/2)-1} sin(2 pi q' d / nx) / q'
  // and the Nyquist mode (even nx) contributes nothing to the real part.
  const double pi = 3.14159265358979323846264338327950288;
  const int qmax = (nx - 1) / 2;
  for (int d = 0; d < nx; ++d) {
    long double acc = 0.0L;
    for (int q = 1; q <= qmax; ++q) {
      const long long r = ((long long)q * d) % nx;
      acc += sinl(2.0L * (long double)pi * (long double)r / (long double)nx) / (long double)q;
    }
    c[d] = (double)(-(long double)length / ((long double)pi * nx) * acc);
  }
  if (hf::poisson_uses_fft(nx)) {  // FFT plan: twiddles exp(-2 pi i m/nx), then 1/k_q
    double *tw = c + nx, *inv_k = c + 2 * nx;
    for (int m = 0; m < nx / 2; ++m) {
      const long double a = -2.0L * (long double)pi * (long double)m / (long double)nx;
      tw[2 * m] = (double)cosl(a);
      tw[2 * m + 1] = (double)sinl(a);
    }
    // k = 2 pi fftfreq(nx, d=dx) (src/baseline_solver.py:26).  The k = 0 mode
    // is zeroed as in the reference; so is the Nyquist mode q = nx/2: for a real
    // rho its term i X/k is purely imaginary, which the reference's Re() drops,
    // and zeroing it lets two ICs share one complex transform (z = rho_a + i
    // rho_b) without that term leaking from one into the other.
    const double dx = length / nx;
    for (int q = 0; q < nx; ++q) {
      const int f = q < (nx + 1) / 2 ? q : q - nx;
      const double k = 2.0 * pi * ((double)f / (nx * dx));
      inv_k[q] = (f == 0 || 2 * q == nx) ? 0.0 : 1.0 / k;
    }
  }
  return HF_OK;
}

int hf_poisson_plan_size(int mode, int nx) {
  if (nx < 1) return -1;
  switch (mode) {
    case HF_POISSON_SPECTRAL: return hf::poisson_plan_len(nx);
    case HF_POISSON_TRIDIAG: return nx <= hf::kTriMaxNx ? 1 : -1;
    default: return -1;
  }
}

int hf_poisson_plan(int mode, int nx, double length, double *plan) {
  if (mode == HF_POISSON_SPECTRAL) return hf_poisson_coeffs(nx, length, plan);
  if (mode != HF_POISSON_TRIDIAG) return fail(HF_EINVAL, "hf_poisson_plan: unknown Poisson mode");
  if (nx < 1 || !(length > 0) || !plan) return fail(HF_EINVAL, "hf_poisson_plan: bad argument");
  if (nx > hf::kTriMaxNx) return fail(HF_EUNSUPPORTED, "hf_poisson_plan: tridiagonal mode needs nx <= 16384");
  plan[0] = 0.5 * (length / nx);  // h = dx/2: E[i] = h (psi[i-1] - psi[i+1]) (hf_device.h)
  return HF_OK;
}

}  // extern "C"

namespace {
// The Poisson mode argument of every *_ex entry point.
int check_mode(int pm, int nx, const char *fn) {
  if (pm != HF_POISSON_SPECTRAL && pm != HF_POISSON_TRIDIAG)
    return fail(HF_EINVAL, std::string(fn) + ": unknown Poisson mode");
  if (!hf::poisson_mode_ok(pm, nx))
    return fail(HF_EUNSUPPORTED, std::string(fn) + ": tridiagonal Poisson needs nx <= 16384");
  return HF_OK;
}
}  // namespace

extern "C" {

int hf_poisson_ex(const float *n, int ld_n, float *E, int ld_E, const double *pc, int pm, int B, int nx,
                  void *stream) {
  if (B < 0 || nx < 1 || ld_n < nx || ld_E < nx) return fail(HF_EINVAL, "hf_poisson: bad shape");
  if (int rc = check_mode(pm, nx, "hf_poisson")) return rc;
  if (B == 0) return HF_OK;
  if (!n || !E || !pc) return fail(HF_EINVAL, "hf_poisson: NULL pointer");
  HF_CHECK_HIP(hf::launch_poisson(n, ld_n, E, ld_E, pc, B, nx, pm, as_stream(stream)), "hf_poisson");
  return HF_OK;
}

int hf_poisson(const float *n, int ld_n, float *E, int ld_E, const double *pc, int B, int nx, void *stream) {
  return hf_poisson_ex(n, ld_n, E, ld_E, pc, HF_POISSON_SPECTRAL, B, nx, stream);
}

int64_t hf_run_workspace_bytes(int op, int B, int nx, int T) {
  if (B < 0 || nx < 1 || T < 0 || op < HF_OP_STEP || op > HF_OP_COMPARE) return -1;
  const int64_t S = 4LL * 3 * nx, F = 4LL * nx, al = 256;
  auto up = [&](int64_t v) { return (v + al - 1) / al * al; };
  switch (op) {
    case HF_OP_STEP: return up(B * F);
    case HF_OP_RUN: return 2 * up(B * S) + up(B * F);
    default: return 2 * up((int64_t)B * (T + 1) * S) + up(B * S) + up(B * F);
  }
}

namespace {

// Scratch for the generic (non-fused) sequencing: carved from the caller's
// workspace when given (hf_run_workspace_bytes), else one stream-ordered
// allocation released on the same stream after the work it backs.
struct Scratch {
  char *base = nullptr;
  bool owned = false;
  int64_t used = 0, cap = 0;
  hipStream_t s = nullptr;
  int init(void *ws, int64_t ws_bytes, int64_t need, hipStream_t st, const char *fn) {
    s = st;
    cap = need;
    if (need == 0) return HF_OK;
    if (ws) {
      if (ws_bytes < need)
        return fail(HF_EINVAL, std::string(fn) + ": workspace smaller than hf_workspace_need");
      base = static_cast<char *>(ws);
      return HF_OK;
    }
    if (hipMallocAsync((void **)&base, need, s) != hipSuccess)
      return fail(HF_ENOMEM, std::string(fn) + ": scratch allocation");
    owned = true;
    return HF_OK;
  }
  float *take(int64_t bytes) {
    float *p = reinterpret_cast<float *>(base + used);
    used += (bytes + 255) / 256 * 256;
    return p;
  }
  ~Scratch() {
    if (owned) (void)hipFreeAsync(base, s);
  }
};

// The per-step sequencing of the generic path for one slice of the batch:
// [chain flux ->] FV + Poisson per step, ping-ponging through buf0/buf1 (or
// the trajectory).  ldT / ldM / ldFT are the per-IC strides of traj, metrics
// and flux_traj, so a slice is the same call on offset pointers.
hipError_t run_steps(const hf_model *m, const float *state0, float *state_final, const float *x, const double *pc,
                     int pm, int B, int nx, int T, float c, float dt, float nu, float dx2, float *traj,
                     float *flux_traj, float *metrics, float *buf0, float *buf1, float *F, hipStream_t s) {
  const int64_t S = 3LL * nx, ldT = (T + 1) * S, ldM = (int64_t)(T + 1) * HF_NUM_METRICS;
  float *buf[2] = {buf0, buf1};
  hipError_t e = hipSuccess;
  const float *cur = state0;
  int64_t ld_cur = S;
  for (int t = 0; t < T && e == hipSuccess; ++t) {
    float *dst;
    int64_t ld_dst;
    if (traj) {
      dst = traj + (int64_t)(t + 1) * S;
      ld_dst = ldT;
    } else if (t == T - 1 && state_final != state0) {
      dst = state_final;
      ld_dst = S;
    } else {
      dst = buf[t & 1];
      ld_dst = S;
    }
    if (m) e = hf::launch_chain_flux(m->chain, nullptr, cur, ld_cur, x, B, nx, nullptr, F, s);
#ifdef HF_DIAG_NOFVSTEP  // timing diagnostic only: results are wrong (hybrid steps launch no FV kernel)
    if (m) {
      cur = dst;
      ld_cur = ld_dst;
      continue;
    }
#endif
    if (e == hipSuccess)
      e = hf::launch_fv_step(cur, ld_cur, dst, ld_dst, F, pc, B, nx, c, dt, nu, dx2,
                             flux_traj ? flux_traj + (int64_t)t * nx : nullptr, (int64_t)T * nx,
                             metrics ? metrics + (int64_t)(t + 1) * HF_NUM_METRICS : nullptr, ldM, pm, s);
    cur = dst;
    ld_cur = ld_dst;
  }
  if (e == hipSuccess && cur != state_final)
    e = hipMemcpy2DAsync(state_final, sizeof(float) * S, cur, sizeof(float) * ld_cur, sizeof(float) * S, B,
                         hipMemcpyDeviceToDevice, s);
  return e;
}

// Lanes of the generic hybrid rollout.  Its steps are a persistent flux kernel
// that fills every CU (one workgroup each, LDS-bound) and then the short
// FV/Poisson kernel; inside one stream the flux kernel's last round of windows
// and the whole FV kernel leave most CUs idle.  With lanes, slices of the
// batch step independently on the caller's stream and on lane streams (forked
// and joined with events), so one slice's flux windows fill the CUs another
// slice's tail and FV leave idle.  Every IC's arithmetic is the same in either
// form.  HF_RUN_LANES=n (1..kMaxLanes) overrides the default (A/B timing).
constexpr int kMaxLanes = 4;
constexpr int kDefaultLanes = 3;  // profiles/r02_lanes_ab.json: 1 / 2 / 3 / 4 lanes = 1.141 / 1.129 / 1.119 / 1.118 ms per cfg4 step
constexpr int64_t kLaneMinCells = 1 << 20;  // each slice still fills the chip for several rounds

// Where hf_run's lanes cut a batch.  The persistent flux kernel of a lane
// runs its units (super-windows) in rounds of one unit per resident
// workgroup, so a lane of u units takes ceil(u / per_round) rounds; slices of
// B/lanes ICs each leave a partly filled last round (cfg4: 3 x 2844 units =
// 3 x 12 rounds of 256 for 33.3 rounds of work), and the lanes' kernels mostly
// run one after another (profiles/r03_v9_bench_kernel_stats.md: the lone
// dispatches take the 12 rounds' time).  When the kernel's units are known,
// every lane but the last gets the most ICs that fill whole rounds (floor of
// the batch's rounds / lanes each: 1352 + 1352 + 1392 ICs = 11 + 11 + 12
// rounds at cfg4), and the last lane the rest; otherwise an even split.
// Which lane steps an IC changes none of its arithmetic.  HF_LANE_CUTS=even
// in the environment selects the even split (A/B timing).
bool lane_cuts_even() {
  static const bool even = [] {
    const char *v = std::getenv("HF_LANE_CUTS");
    return v && std::strcmp(v, "even") == 0;
  }();
  return even;
}
void lane_cuts(const hf_model *m, int B, int nx, int lanes, int64_t *cut) {
  for (int i = 0; i <= lanes; ++i) cut[i] = (int64_t)B * i / lanes;
  if (!m || lanes < 2 || lane_cuts_even()) return;
  const hf::FluxWork all = hf::chain_flux_work(m->chain, B, nx);
  if (all.per_round <= 0) return;
  const int64_t k = all.units / all.per_round / lanes;  // whole rounds per leading lane
  if (k < 1) return;
  // computed whole into a local set, copied over the even split only when every lane is placed
  int64_t c[kMaxLanes + 1] = {0};
  int64_t o = 0;
  for (int i = 0; i + 1 < lanes; ++i) {
    // the most ICs whose units fit k rounds (units grow by at most
    // ceil(P / faces) per IC, so step down from the even share's estimate)
    int64_t n = (int64_t)B / lanes + 1;
    while (n > 1 && hf::chain_flux_work(m->chain, n, nx).units > k * all.per_round) --n;
    if (o + n >= B) return;  // keep the even split: nothing left for the last lane
    c[i + 1] = o += n;
  }
  c[lanes] = B;
  for (int i = 0; i <= lanes; ++i) cut[i] = c[i];
}

int run_lanes() {
  static const int lanes = [] {
    const char *v = std::getenv("HF_RUN_LANES");
    const int n = v ? std::atoi(v) : kDefaultLanes;
    return n < 1 ? 1 : n > kMaxLanes ? kMaxLanes : n;
  }();
  return lanes;
}

// The classical rollout at FFT sizes runs as one persistent launch
// (fv_run_fft_kernel); HF_FV_PERSIST=0 in the environment selects the
// per-step launches instead (A/B timing and the bitwise equality test only).
bool fv_run_persistent() {
  static const bool on = [] {
    const char *v = std::getenv("HF_FV_PERSIST");
    return !(v && v[0] == '0');
  }();
  return on;
}

int64_t up256(int64_t v) { return (v + 255) / 256 * 256; }

// The scratch each path actually carves (hf_workspace_need): the fused
// rollouts and the one-launch classical rollouts take none; the generic run
// takes two state buffers unless the trajectory is the ping-pong, plus the
// face flux of the hybrid step; the FFT compare one hybrid trajectory and the
// flux; the generic compare both trajectories, a state and the flux.
int64_t need_step(const hf_model *m, int B, int nx, bool has_ff) {
  if (!m || fused_nx(nx) || has_ff) return 0;
  return up256(4LL * B * nx);
}
int64_t need_run(const hf_model *m, int B, int nx, int T, bool has_traj) {
  if (B == 0 || T == 0 || (m && fused_nx(nx))) return 0;
  if (!m && hf::fv_run_fused(nx) && fv_run_persistent()) return 0;
  return (has_traj ? 0 : 2 * up256(12LL * B * nx)) + (m ? up256(4LL * B * nx) : 0);
}
bool compare_fft_twin(int nx) { return hf::poisson_uses_fft(nx) && hf::fv_run_fused(nx) && fv_run_persistent(); }
int64_t need_compare(int B, int nx, int T) {
  if (B == 0 || fused_nx(nx)) return 0;
  const int64_t traj = up256(12LL * B * (T + 1) * nx), flux = up256(4LL * B * nx);
  if (compare_fft_twin(nx)) return traj + flux;
  return 2 * traj + up256(12LL * B * nx) + flux;
}

// Lane streams belong to the caller's stream: lane i (1..kMaxLanes-1) of
// (current device, caller stream), created on first use.  Calls on different
// caller streams (other threads, other streams of one thread) therefore never
// share a lane, so they do not serialise through each other's lanes, and a
// graph capture of one caller stream pulls only that stream's own lanes into
// capture mode.  Calls on one caller stream are ordered by that stream anyway.
// At most kMaxLaneOwners caller streams get lanes; later ones run one lane.
constexpr int kMaxLaneOwners = 256;

struct LaneSet {
  int dev;
  hipStream_t owner;
  hipStream_t lane[kMaxLanes];
};

hipError_t lane_streams(hipStream_t caller, int lanes, hipStream_t *out, bool *granted) {
  static std::mutex mu;
  static std::vector<LaneSet> sets;
  *granted = false;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lock(mu);
  LaneSet *ls = nullptr;
  for (auto &x : sets)
    if (x.dev == dev && x.owner == caller) ls = &x;
  if (!ls) {
    if ((int)sets.size() >= kMaxLaneOwners) return hipSuccess;
    sets.push_back(LaneSet{dev, caller, {}});
    ls = &sets.back();
  }
  for (int i = 1; i < lanes; ++i) {
    if (!ls->lane[i]) {
      e = hipStreamCreateWithFlags(&ls->lane[i], hipStreamNonBlocking);
      if (e != hipSuccess) return e;
    }
    out[i] = ls->lane[i];
  }
  *granted = true;
  return hipSuccess;
}

}  // namespace

int64_t hf_workspace_need(hf_model_t m, int op, int B, int nx, int T, int flags) {
  if (B < 0 || nx < 1 || T < 0 || op < HF_OP_STEP || op > HF_OP_COMPARE) return -1;
  if (flags & ~(HF_WS_TRAJ | HF_WS_FLUX_FACE)) return -1;
  switch (op) {
    case HF_OP_STEP: return need_step(m, B, nx, flags & HF_WS_FLUX_FACE);
    case HF_OP_RUN: return need_run(m, B, nx, T, flags & HF_WS_TRAJ);
    default: return m ? need_compare(B, nx, T) : -1;
  }
}

int hf_step_ex(hf_model_t m, const float *in, float *out, const float *x, const double *pc, int pm, int B, int nx,
               float c, float dt, float nu, float dx2, float *ff, float *metrics, void *ws, int64_t ws_bytes,
               void *stream) {
  if (B < 0 || nx < 1) return fail(HF_EINVAL, "hf_step: need B >= 0, nx >= 1");
  if (int rc = check_mode(pm, nx, "hf_step")) return rc;
  if (B == 0) return HF_OK;
  if (!in || !out || !pc) return fail(HF_EINVAL, "hf_step: NULL state or Poisson coefficients");
  if (in == out) return fail(HF_EINVAL, "hf_step: state_in and state_out must not alias");
  hipStream_t s = as_stream(stream);
  if (!m) {  // BaselineSolver.step
    HF_CHECK_HIP(hf::launch_fv_step(in, 3LL * nx, out, 3LL * nx, nullptr, pc, B, nx, c, dt, nu, dx2, ff,
                                    nx, metrics, HF_NUM_METRICS, pm, s),
                 "hf_step(classical)");
    return HF_OK;
  }
  if (!x) return fail(HF_EINVAL, "hf_step: NULL x");
  if (int rc = chain_usable(m)) return rc;
  if (fused_nx(nx)) {
    hf::RolloutExtras ex;
    ex.poisson = pm;
    HF_CHECK_HIP(hf::launch_chain_rollout(m->chain, in, out, x, pc, B, nx, 1, c, dt, nullptr, ff, nullptr, s, ex),
                 "hf_step(hybrid fused)");
    if (metrics)
      HF_CHECK_HIP(hf::launch_state_metrics(out, 3LL * nx, B, nx, metrics, HF_NUM_METRICS, s), "hf_step metrics");
    return HF_OK;
  }
  Scratch sc;
  if (int rc = sc.init(ws, ws_bytes, need_step(m, B, nx, ff != nullptr), s, "hf_step"))
    return rc;
  float *F = ff ? ff : sc.take(sizeof(float) * (int64_t)B * nx);
  HF_CHECK_HIP(hf::launch_chain_flux(m->chain, nullptr, in, 3LL * nx, x, B, nx, nullptr, F, s), "hf_step(flux)");
  HF_CHECK_HIP(hf::launch_fv_step(in, 3LL * nx, out, 3LL * nx, F, pc, B, nx, c, dt, nu, dx2, nullptr, nx, metrics,
                                  HF_NUM_METRICS, pm, s),
               "hf_step(fv)");
  return HF_OK;
}

int hf_step(hf_model_t m, const float *in, float *out, const float *x, const double *pc, int B, int nx, float c,
            float dt, float nu, float dx2, float *ff, float *metrics, void *ws, int64_t ws_bytes, void *stream) {
  return hf_step_ex(m, in, out, x, pc, HF_POISSON_SPECTRAL, B, nx, c, dt, nu, dx2, ff, metrics, ws, ws_bytes,
                    stream);
}

int hf_run_ex(hf_model_t m, const float *state0, float *state_final, const float *x, const double *pc, int pm,
              int B, int nx, int T, float c, float dt, float nu, float dx2, float *traj, float *flux_traj,
              float *metrics, void *ws, int64_t ws_bytes, void *stream) {
  if (B < 0 || nx < 1 || T < 0) return fail(HF_EINVAL, "hf_run: need B >= 0, nx >= 1, T >= 0");
  if (int rc = check_mode(pm, nx, "hf_run")) return rc;
  if (B == 0) return HF_OK;
  if (!state0 || !state_final || !pc) return fail(HF_EINVAL, "hf_run: NULL state or Poisson coefficients");
  if (m && !x) return fail(HF_EINVAL, "hf_run: NULL x");
  if (m) {
    if (int rc = chain_usable(m)) return rc;
  }
  hipStream_t s = as_stream(stream);
  const int64_t S = 3LL * nx;  // floats per state
  if (m && fused_nx(nx)) {  // the kernel reads each IC's state0 whole before writing its state_final
    hf::RolloutExtras ex;
    ex.poisson = pm;
    HF_CHECK_HIP(hf::launch_chain_rollout(m->chain, state0, state_final, x, pc, B, nx, T, c, dt, traj,
                                          flux_traj, metrics, s, ex),
                 "hf_run(hybrid fused)");
    return HF_OK;
  }
  // Generic sequencing: [chain flux ->] FV+Poisson per step, ping-ponging
  // through scratch (or the trajectory); state0 may alias state_final.
  const int64_t ldT = (T + 1) * S, ldM = (int64_t)(T + 1) * HF_NUM_METRICS;
  if (traj)
    HF_CHECK_HIP(hipMemcpy2DAsync(traj, sizeof(float) * ldT, state0, sizeof(float) * S, sizeof(float) * S, B,
                                  hipMemcpyDeviceToDevice, s),
                 "hf_run traj[0]");
  if (metrics) HF_CHECK_HIP(hf::launch_state_metrics(state0, S, B, nx, metrics, ldM, s), "hf_run metrics[0]");
  if (T == 0) {
    if (state_final != state0)
      HF_CHECK_HIP(hipMemcpyAsync(state_final, state0, sizeof(float) * B * S, hipMemcpyDeviceToDevice, s),
                   "hf_run copy");
    return HF_OK;
  }
  if (!m && hf::fv_run_fused(nx) && fv_run_persistent()) {  // BaselineSolver.run at FFT nx <= 1024 and nx <= 64: one launch
    HF_CHECK_HIP(hf::launch_fv_run(state0, S, state_final, traj, pc, B, nx, T, c, dt, nu, dx2, flux_traj, metrics,
                                   nullptr, nullptr, pm, s),
                 "hf_run(classical fused)");
    return HF_OK;
  }
  // scratch: two state buffers unless the trajectory is the ping-pong, the face flux for the hybrid step
  const int64_t sbytes = (sizeof(float) * B * S + 255) / 256 * 256, fbytes = (sizeof(float) * B * nx + 255) / 256 * 256;
  Scratch sc;
  if (int rc = sc.init(ws, ws_bytes, need_run(m, B, nx, T, traj != nullptr), s, "hf_run")) return rc;
  float *buf0 = nullptr, *buf1 = nullptr;
  if (!traj) buf0 = sc.take(sbytes), buf1 = sc.take(sbytes);
  float *F = m ? sc.take(fbytes) : nullptr;
  int lanes = run_lanes();
  while (lanes > 1 && (int64_t)B * nx < lanes * kLaneMinCells) --lanes;
  if (!m || B < lanes) lanes = 1;
  if (lanes > 1 && s) {  // lane streams live on the current device: a stream of another device runs one lane
    int cur = 0;
    hipDevice_t sdev = 0;
    if (hipGetDevice(&cur) != hipSuccess || hipStreamGetDevice(s, &sdev) != hipSuccess || sdev != cur) lanes = 1;
  }
  if (lanes == 1) {
    HF_CHECK_HIP(run_steps(m, state0, state_final, x, pc, pm, B, nx, T, c, dt, nu, dx2, traj, flux_traj, metrics,
                           buf0, buf1, F, s),
                 "hf_run");
    return HF_OK;
  }
  // lane i steps ICs [cut[i], cut[i+1]); lane 0 on the caller's stream
  int64_t cut[kMaxLanes + 1];
  lane_cuts(m, B, nx, lanes, cut);
  hipStream_t ls[kMaxLanes] = {s};
  bool granted = false;
  HF_CHECK_HIP(lane_streams(s, lanes, ls, &granted), "hf_run lane stream");
  if (!granted) {
    HF_CHECK_HIP(run_steps(m, state0, state_final, x, pc, pm, B, nx, T, c, dt, nu, dx2, traj, flux_traj, metrics,
                           buf0, buf1, F, s),
                 "hf_run");
    return HF_OK;
  }
  hipEvent_t fork = nullptr, join[kMaxLanes] = {};
  for (int i = 1; i < lanes; ++i) {
    hipError_t ce = hipEventCreateWithFlags(&join[i], hipEventDisableTiming);
    if (ce != hipSuccess) {
      for (int k = 1; k < i; ++k) (void)hipEventDestroy(join[k]);
      return fail_hip(ce, "hf_run lane event");
    }
  }
  hipError_t e = hipEventCreateWithFlags(&fork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(fork, s);
  bool used[kMaxLanes] = {};  // lane streams that received work
  for (int i = lanes - 1; i >= 0 && e == hipSuccess; --i) {
    const int64_t o = cut[i], n = cut[i + 1] - o;
    if (i > 0) e = hipStreamWaitEvent(ls[i], fork, 0);
    if (e != hipSuccess) break;
    used[i] = true;
    e = run_steps(m, state0 + o * S, state_final + o * S, x, pc, pm, (int)n, nx, T, c, dt, nu, dx2,
                  traj ? traj + o * ldT : nullptr, flux_traj ? flux_traj + o * T * nx : nullptr,
                  metrics ? metrics + o * ldM : nullptr, buf0 ? buf0 + o * S : nullptr,
                  buf1 ? buf1 + o * S : nullptr, F + o * nx, ls[i]);
  }
  // join every lane that received work, also after an error, so that nothing
  // enqueued on a lane outlives the call's scratch (freed on `s`) unordered
  for (int i = 1; i < lanes; ++i) {
    if (!used[i]) continue;
    hipError_t je = hipEventRecord(join[i], ls[i]);
    if (je == hipSuccess) je = hipStreamWaitEvent(s, join[i], 0);
    if (je != hipSuccess) (void)hipStreamSynchronize(ls[i]);
    if (e == hipSuccess) e = je;
  }
  if (fork) (void)hipEventDestroy(fork);
  for (int i = 1; i < lanes; ++i)
    if (join[i]) (void)hipEventDestroy(join[i]);
  HF_CHECK_HIP(e, "hf_run");
  return HF_OK;
}

int hf_run(hf_model_t m, const float *state0, float *state_final, const float *x, const double *pc, int B, int nx,
           int T, float c, float dt, float nu, float dx2, float *traj, float *flux_traj, float *metrics, void *ws,
           int64_t ws_bytes, void *stream) {
  return hf_run_ex(m, state0, state_final, x, pc, HF_POISSON_SPECTRAL, B, nx, T, c, dt, nu, dx2, traj, flux_traj,
                   metrics, ws, ws_bytes, stream);
}

int hf_run_compare_ex(hf_model_t m, const float *state0, float *state_final, const float *x, const double *pc, int pm,
                      int B, int nx, int T, float c, float dt, float nu, float dx2, float *mse, float *metrics,
                      float *metrics_cl, void *ws, int64_t ws_bytes, void *stream) {
  if (!m) return fail(HF_EINVAL, "hf_run_compare: NULL model");
  if (B < 0 || nx < 1 || T < 0) return fail(HF_EINVAL, "hf_run_compare: need B >= 0, nx >= 1, T >= 0");
  if (int rc = check_mode(pm, nx, "hf_run_compare")) return rc;
  if (B == 0) return HF_OK;
  if (!state0 || !state_final || !pc || !x || !mse) return fail(HF_EINVAL, "hf_run_compare: NULL pointer");
  if (int rc = chain_usable(m)) return rc;
  hipStream_t s = as_stream(stream);
  if (fused_nx(nx)) {
    hf::RolloutExtras ex;
    ex.nu = nu;
    ex.dx2 = dx2;
    ex.mse = mse;
    ex.metrics_cl = metrics_cl;
    ex.poisson = pm;
    HF_CHECK_HIP(hf::launch_chain_rollout(m->chain, state0, state_final, x, pc, B, nx, T, c, dt, nullptr, nullptr,
                                          metrics, s, ex),
                 "hf_run_compare(fused)");
    return HF_OK;
  }
  if (compare_fft_twin(nx)) {
    // FFT nx <= 1024: the hybrid rollout first, recording its trajectory; then
    // the classical twin as one launch from that trajectory's row 0 (state0,
    // also when state_final aliases it), scoring each step against the hybrid
    // row as it goes: no classical trajectory, no MSE pass.  Same bits as below.
    Scratch sc;
    if (int rc = sc.init(ws, ws_bytes, need_compare(B, nx, T), s, "hf_run_compare"))
      return rc;
    const int64_t S = 3LL * nx, ldT = (T + 1) * S;
    float *th = sc.take(sizeof(float) * (int64_t)B * ldT);
    const int64_t fbytes = (sizeof(float) * (int64_t)B * nx + 255) / 256 * 256;
    float *F = sc.take(fbytes);
    int rc =
        hf_run_ex(m, state0, state_final, x, pc, pm, B, nx, T, c, dt, nu, dx2, th, nullptr, metrics, F, fbytes, stream);
    if (rc != HF_OK) return rc;
    if (metrics_cl)
      HF_CHECK_HIP(hf::launch_state_metrics(th, ldT, B, nx, metrics_cl, (int64_t)(T + 1) * HF_NUM_METRICS, s),
                   "hf_run_compare metrics[0]");
    HF_CHECK_HIP(hf::launch_fv_run(th, ldT, nullptr, nullptr, pc, B, nx, T, c, dt, nu, dx2, nullptr, metrics_cl, th, mse,
                                   pm, s),
                 "hf_run_compare(classical twin)");
    return HF_OK;
  }
  // generic nx: both trajectories through HBM, then the MSE reduction.  The
  // classical twin runs first: state_final may alias state0, and the hybrid
  // run is the one that writes it.
  Scratch sc;
  if (int rc = sc.init(ws, ws_bytes, need_compare(B, nx, T), s, "hf_run_compare"))
    return rc;
  const int64_t traj_bytes = sizeof(float) * (int64_t)B * (T + 1) * 3 * nx;
  float *th = sc.take(traj_bytes), *tc = sc.take(traj_bytes), *fin_c = sc.take(sizeof(float) * (int64_t)B * 3 * nx);
  const int64_t fbytes = (sizeof(float) * (int64_t)B * nx + 255) / 256 * 256;
  float *F = sc.take(fbytes);
  // with a trajectory buffer hf_run needs scratch only for the hybrid face flux
  int rc = hf_run_ex(nullptr, state0, fin_c, x, pc, pm, B, nx, T, c, dt, nu, dx2, tc, nullptr, metrics_cl, nullptr, 0,
                     stream);
  if (rc == HF_OK)
    rc = hf_run_ex(m, state0, state_final, x, pc, pm, B, nx, T, c, dt, nu, dx2, th, nullptr, metrics, F, fbytes,
                   stream);
  if (rc != HF_OK) return rc;
  HF_CHECK_HIP(hf::launch_traj_mse(th, tc, B, T + 1, nx, mse, s), "hf_run_compare mse");
  return HF_OK;
}

int hf_run_compare(hf_model_t m, const float *state0, float *state_final, const float *x, const double *pc, int B,
                   int nx, int T, float c, float dt, float nu, float dx2, float *mse, float *metrics,
                   float *metrics_cl, void *ws, int64_t ws_bytes, void *stream) {
  return hf_run_compare_ex(m, state0, state_final, x, pc, HF_POISSON_SPECTRAL, B, nx, T, c, dt, nu, dx2, mse,
                           metrics, metrics_cl, ws, ws_bytes, stream);
}

int hf_traj_metrics(const float *traj, int B, int T1, int nx, float *metrics, void *stream) {
  if (B < 0 || T1 < 0 || nx < 1) return fail(HF_EINVAL, "hf_traj_metrics: bad shape");
  if ((int64_t)B * T1 == 0) return HF_OK;
  if (!traj || !metrics) return fail(HF_EINVAL, "hf_traj_metrics: NULL pointer");
  if ((int64_t)B * T1 > 0x7fffffffLL) return fail(HF_EUNSUPPORTED, "hf_traj_metrics: > 2^31 states");
  HF_CHECK_HIP(hf::launch_state_metrics(traj, 3LL * nx, B * T1, nx, metrics, HF_NUM_METRICS, as_stream(stream)),
               "hf_traj_metrics");
  return HF_OK;
}

int hf_traj_mse(const float *a, const float *b, int B, int T1, int nx, float *mse, void *stream) {
  if (B < 0 || T1 < 0 || nx < 1) return fail(HF_EINVAL, "hf_traj_mse: bad shape");
  if ((int64_t)B * T1 == 0) return HF_OK;
  if (!a || !b || !mse) return fail(HF_EINVAL, "hf_traj_mse: NULL pointer");
  HF_CHECK_HIP(hf::launch_traj_mse(a, b, B, T1, nx, mse, as_stream(stream)), "hf_traj_mse");
  return HF_OK;
}

int hf_rollout_summary(const float *metrics, const float *mse, const float *metrics_ref, int B, int T,
                       float *summary, float *drift, void *stream) {
  if (B < 0 || T < 0) return fail(HF_EINVAL, "hf_rollout_summary: need B >= 0, T >= 0");
  if (B == 0) return HF_OK;
  if (!metrics || !summary) return fail(HF_EINVAL, "hf_rollout_summary: NULL metrics or summary");
  HF_CHECK_HIP(hf::launch_rollout_summary(metrics, mse, metrics_ref, B, T, summary, drift, as_stream(stream)),
               "hf_rollout_summary");
  return HF_OK;
}

}  // extern "C"
