// Host-sanitized drive of the C ABI (SURVEY.md §5 "bounds-checked debug build").
//
// Built by `make -C gnn-plasma-flux_amd/csrc asan` with AddressSanitizer and
// UBSan on the HOST code only (weight packing, argument checks, plan building,
// workspace arithmetic, lane fork/join); device code is the normal gfx950
// build.  Without a device it runs the host-only entry points and the
// argument checks; with one it also runs every rollout path once at a small
// size (fused, cell-split, windowed, FFT, circulant, classical one-launch,
// compare, scoring) and checks return codes and finiteness.  Exit 0 = clean.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hybridflux.h"

static int g_fail = 0;
#define EXPECT(cond)                                                   \
  do {                                                                 \
    if (!(cond)) {                                                     \
      std::fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond, hf_last_error()); \
      ++g_fail;                                                        \
    }                                                                  \
  } while (0)

static float lcg(unsigned &s) {
  s = s * 1664525u + 1013904223u;
  return ((s >> 8) & 0xFFFF) / 65536.0f - 0.5f;
}

struct Dev {
  void *p = nullptr;
  explicit Dev(size_t bytes) {
    if (hipMalloc(&p, bytes ? bytes : 4) != hipSuccess) std::abort();
    (void)hipMemset(p, 0, bytes ? bytes : 4);
  }
  ~Dev() { (void)hipFree(p); }
  float *f() const { return static_cast<float *>(p); }
  double *d() const { return static_cast<double *>(p); }
};

static void host_only() {
  EXPECT(hf_version() != nullptr);
  EXPECT(hf_model_param_count(4, 128, 4) == 165249);
  EXPECT(hf_model_param_count(0, 128, 4) == -1);
  for (int nx : {1, 2, 3, 16, 63, 64, 100, 255, 256, 512, 1024, 2048, 4096, 6145, 8192}) {
    const int len = hf_poisson_plan_len(nx);
    EXPECT(len >= nx);
    std::vector<double> c((size_t)len);  // exact size: an overrun is an ASan report
    EXPECT(hf_poisson_coeffs(nx, 2 * M_PI, c.data()) == HF_OK);
    for (double v : c) EXPECT(std::isfinite(v));
  }
  EXPECT(hf_poisson_plan_len(0) < 0);
  EXPECT(hf_poisson_coeffs(0, 1.0, nullptr) != HF_OK);
  for (int op : {HF_OP_STEP, HF_OP_RUN, HF_OP_COMPARE}) {
    EXPECT(hf_run_workspace_bytes(op, 32768, 1024, 100000) > 0);  // no int overflow (UBSan)
    EXPECT(hf_run_workspace_bytes(op, -1, 64, 1) == -1);
  }
  EXPECT(hf_run_workspace_bytes(7, 1, 64, 1) == -1);
  float dummy[4] = {};
  hf_model_t m = nullptr;
  EXPECT(hf_model_create(nullptr, 4, 128, 4, HF_WDTYPE_F32, &m) == HF_EINVAL);
  EXPECT(hf_model_create(dummy, 4, 128, 4, 9, &m) == HF_EINVAL);
  EXPECT(hf_model_create(dummy, 4, 128, 4, HF_WDTYPE_F32, nullptr) == HF_EINVAL);
  EXPECT(hf_run(nullptr, nullptr, nullptr, nullptr, nullptr, 4, 64, 3, 0, 0, 0, 0, nullptr, nullptr, nullptr,
                nullptr, 0, nullptr) == HF_EINVAL);
  EXPECT(hf_run(nullptr, dummy, dummy, nullptr, nullptr, -1, 64, 3, 0, 0, 0, 0, nullptr, nullptr, nullptr, nullptr, 0,
                nullptr) == HF_EINVAL);
  EXPECT(hf_step(nullptr, dummy, dummy, nullptr, nullptr, 1, 64, 0, 0, 0, 0, nullptr, nullptr, nullptr, 0, nullptr) ==
         HF_EINVAL);
}

// one rollout of every kind at B ICs x nx cells; expects finite final states
static void rollouts(hf_model_t m, int B, int nx, int T) {
  const int64_t S = 3LL * nx;
  const double L = 2 * M_PI, dx = L / nx, dtd = 5e-3 * 64 / (nx < 64 ? 64 : nx);
  const float c = (float)(dtd / dx), dt = (float)dtd, nu = 1e-3f, dx2 = (float)(dx * dx);
  std::vector<float> h((size_t)(B * S)), x((size_t)nx);
  for (int i = 0; i < nx; ++i) x[i] = (float)((i + 0.5) * dx);
  for (int b = 0; b < B; ++b)
    for (int i = 0; i < nx; ++i) {
      h[b * S + i] = 1.f + 0.01f * std::sin((b + 1) * x[i]);
      h[b * S + nx + i] = 0.01f * std::cos((b + 2) * x[i]);
      h[b * S + 2 * nx + i] = 0.f;
    }
  std::vector<double> plan((size_t)hf_poisson_plan_len(nx));
  EXPECT(hf_poisson_coeffs(nx, L, plan.data()) == HF_OK);
  Dev st(4 * h.size()), fin(4 * h.size()), dx_(4 * x.size()), pc(8 * plan.size());
  Dev traj(4 * (size_t)B * (T + 1) * S), flux(4 * (size_t)B * T * nx), met(16 * (size_t)B * (T + 1)),
      met2(16 * (size_t)B * (T + 1)), mse(12 * (size_t)B * (T + 1)), summ(4 * 64 * (size_t)B),
      drift(16 * (size_t)B * (T + 1));
  (void)hipMemcpy(st.p, h.data(), 4 * h.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(dx_.p, x.data(), 4 * x.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(pc.p, plan.data(), 8 * plan.size(), hipMemcpyHostToDevice);
  EXPECT(hf_poisson(st.f(), (int)S, st.f() + 2 * nx, (int)S, pc.d(), B, nx, nullptr) == HF_OK);
  EXPECT(hf_run(m, st.f(), fin.f(), dx_.f(), pc.d(), B, nx, T, c, dt, nu, dx2, traj.f(), flux.f(), met.f(), nullptr,
                0, nullptr) == HF_OK);
  EXPECT(hf_run(m, st.f(), fin.f(), dx_.f(), pc.d(), B, nx, T, c, dt, nu, dx2, nullptr, nullptr, nullptr, nullptr, 0,
                nullptr) == HF_OK);
  EXPECT(hf_step(m, st.f(), fin.f(), dx_.f(), pc.d(), B, nx, c, dt, nu, dx2, flux.f(), met.f(), nullptr, 0,
                 nullptr) == HF_OK);
  if (m) {
    EXPECT(hf_run_compare(m, st.f(), fin.f(), dx_.f(), pc.d(), B, nx, T, c, dt, nu, dx2, mse.f(), met.f(), met2.f(),
                          nullptr, 0, nullptr) == HF_OK);
    EXPECT(hf_rollout_summary(met.f(), mse.f(), met2.f(), B, T, summ.f(), drift.f(), nullptr) == HF_OK);
  }
  EXPECT(hf_traj_metrics(traj.f(), B, T + 1, nx, met.f(), nullptr) == HF_OK);
  EXPECT(hipDeviceSynchronize() == hipSuccess);
  std::vector<float> out(h.size());
  (void)hipMemcpy(out.data(), fin.p, 4 * out.size(), hipMemcpyDeviceToHost);
  bool finite = true;
  for (float v : out) finite &= std::isfinite(v);
  if (!finite) std::fprintf(stderr, "non-finite final state: model=%p B=%d nx=%d\n", (void *)m, B, nx);
  EXPECT(finite);
}

int main() {
  host_only();
  int ndev = hf_device_count();
  std::printf("host-only checks done (%d failures); devices: %d; %s\n", g_fail, ndev, hf_version());
  if (ndev > 0) {
    const int64_t P = hf_model_param_count(4, 128, 4);
    std::vector<float> params((size_t)P);
    unsigned seed = 12345;
    for (float &v : params) v = 0.05f * lcg(seed);
    for (int wd : {HF_WDTYPE_F32, HF_WDTYPE_BF16, HF_WDTYPE_F16X3}) {
      hf_model_t m = nullptr;
      EXPECT(hf_model_create(params.data(), 4, 128, 4, wd, &m) == HF_OK);
      for (int nx : {64, 32, 100, 256})
        for (int B : {3, 600}) rollouts(m, B, nx, 4);
      hf_model_destroy(m);
    }
    for (int nx : {64, 100, 256, 1024}) rollouts(nullptr, 5, nx, 4);  // classical: circulant, FFT one-launch
    std::printf("device checks done\n");
  }
  std::printf("%s: %d failures\n", g_fail ? "FAILED" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
