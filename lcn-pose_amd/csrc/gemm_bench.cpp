// Stand-alone timing of the block-sparse GEMM kernels at the cfg3 shape
// (B = 65 536, F = 64, knn = 3: 175 blocks), random data, HIP events.
// Build: make gemm_bench ; run: ./gemm_bench [B] [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <random>
#include <vector>

#include "lcn_internal.h"

using namespace lcn;

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

static const int kNbr[17][7] = {{1, 4, 7, -1}, {0, 7, 2, -1}, {1, 3, -1}, {2, -1}, {0, 7, 5, -1},
                                {4, 6, -1}, {5, -1}, {1, 0, 4, 14, 8, 11, -1}, {7, 9, 11, 14, -1},
                                {8, 10, -1}, {9, -1}, {8, 7, 12, -1}, {11, 13, -1}, {12, -1},
                                {8, 7, 15, -1}, {14, 16, -1}, {15, -1}};

template <typename T>
T* dev(const std::vector<T>& v) {
  T* p;
  CK(hipMalloc(&p, v.size() * sizeof(T)));
  CK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? std::atoi(argv[1]) : 65536;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 20;
  const int knn = argc > 3 ? std::atoi(argv[3]) : 3;
  const int J = 17, F = 64, H = J * F;
  // structure N = (A+I)^knn != 0
  std::vector<int> A(J * J, 0);
  for (int i = 0; i < J; ++i) {
    A[i * J + i] = 1;
    for (int k = 0; kNbr[i][k] >= 0; ++k) A[i * J + kNbr[i][k]] = 1;
  }
  std::vector<int> N = A;
  for (int p = 1; p < knn; ++p) {
    std::vector<int> T(J * J, 0);
    for (int i = 0; i < J; ++i)
      for (int j = 0; j < J; ++j)
        for (int k = 0; k < J; ++k) T[i * J + j] |= N[i * J + k] && A[k * J + j];
    N = T;
  }
  std::vector<int2> blk;
  std::vector<int> bid(J * J, -1);
  for (int i = 0; i < J; ++i)
    for (int j = 0; j < J; ++j)
      if (N[j * J + i]) { bid[i * J + j] = (int)blk.size(); blk.push_back(make_int2(i, j)); }
  std::vector<int> fptr(1, 0), bptr(1, 0);
  std::vector<int2> fidx, bidx;
  for (int so = 0; so < J; ++so) {
    for (int si = 0; si < J; ++si)
      if (bid[si * J + so] >= 0) fidx.push_back(make_int2(si, bid[si * J + so]));
    fptr.push_back((int)fidx.size());
  }
  for (int si = 0; si < J; ++si) {
    for (int so = 0; so < J; ++so)
      if (bid[si * J + so] >= 0) bidx.push_back(make_int2(so, bid[si * J + so]));
    bptr.push_back((int)bidx.size());
  }
  const int nblk = (int)blk.size();
  std::printf("B=%d knn=%d nblk=%d\n", B, knn, nblk);
  if (std::getenv("LCN_LIST_ORDER")) {  // entries of every list by falling popularity of the input slab
    const int mode = std::atoi(std::getenv("LCN_LIST_ORDER"));
    auto reorder = [&](const std::vector<int>& ptr, std::vector<int2>& idx) {
      std::vector<int> pop(J, 0);
      for (const int2& e : idx) pop[e.x]++;
      for (int so = 0; so < J; ++so)
        std::stable_sort(idx.begin() + ptr[so], idx.begin() + ptr[so + 1], [&](const int2& x, const int2& y) {
          return mode == 1 ? pop[x.x] > pop[y.x] : pop[x.x] < pop[y.x];
        });
    };
    reorder(fptr, fidx);
    reorder(bptr, bidx);
  }

  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  std::vector<float> hx((size_t)B * H), hw((size_t)nblk * 4096), hb(H), hs(F), hh(F);
  for (auto& v : hx) v = U(rng);
  for (auto& v : hw) v = U(rng) * 0.05f;
  for (auto& v : hb) v = U(rng);
  for (int f = 0; f < F; ++f) { hs[f] = 1.f + 0.1f * U(rng); hh[f] = 0.1f * U(rng); }
  float* X = dev(hx);
  float* X2 = dev(hx);
  float* W = dev(hw);
  float* bias = dev(hb);
  float* sc = dev(hs);
  float* sh = dev(hh);
  std::vector<float> hc(3 * F), hm(F, 0.f), hr(F, 1.f);
  for (int f = 0; f < F; ++f) { hc[f] = 1.f; hc[F + f] = 0.01f * U(rng); hc[2 * F + f] = 0.01f * U(rng); }
  float* c123 = dev(hc);
  float* mean = dev(hm);
  float* rstd = dev(hr);
  int2* dblk = dev(blk);
  int* dfp = dev(fptr);
  int* dbp = dev(bptr);
  int2* dfi = dev(fidx);
  int2* dbi = dev(bidx);
  auto by_length = [&](const std::vector<int>& ptr) {
    std::vector<int> o(J);
    for (int i = 0; i < J; ++i) o[i] = i;
    std::stable_sort(o.begin(), o.end(), [&](int x, int y) { return ptr[x + 1] - ptr[x] > ptr[y + 1] - ptr[y]; });
    return o;
  };
  int* dfo = dev(by_length(fptr));
  int* dbo = dev(by_length(bptr));
  const int tail = std::getenv("LCN_GEMM_TAIL") ? std::atoi(std::getenv("LCN_GEMM_TAIL")) : 16;
  // variant 1: two output slabs per workgroup (gemm_pair.hip)
  const PairPlan fpp = make_pair_plan(fptr, fidx, J), bpp = make_pair_plan(bptr, bidx, J);
  int4 *dfpp = dev(fpp.pairs), *dbpp = dev(bpp.pairs), *dfpm = dev(fpp.ment), *dbpm = dev(bpp.ment);
  int *dfpo = dev(fpp.order), *dbpo = dev(bpp.order);
  std::printf("pairs: %zu forward (%d of %d activation loads saved), %zu backward (%d saved)\n", fpp.pairs.size(), fpp.saved,
              nblk, bpp.pairs.size(), bpp.saved);
  float* Y;
  CK(hipMalloc(&Y, (size_t)B * H * 4));
  float2* stat;
  CK(hipMalloc(&stat, (size_t)(B / 32 + 1) * H * 8 + (size_t)B * 17));
  const int nch = std::getenv("LCN_DW_NCH") ? std::atoi(std::getenv("LCN_DW_NCH")) : std::max(1, std::min(64, 5600 / nblk));
  float* part;
  CK(hipMalloc(&part, (size_t)128 * nblk * 4096 * 4));
  float* dW;
  CK(hipMalloc(&dW, (size_t)H * H * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double flop = 2.0 * 4096.0 * nblk * B;

  // kind 0: forward (bias, EPI_BNFWD); 1: backward-data (+residual, EPI_BNBACK)
  // kind 3: forward without epilogue partials; 4: same with every row reading
  // row 0 of X (ldx = 0: operand traffic all cache hits -- the in-core ceiling)
  auto mk = [&](int kind, int pro, int variant) {
    const bool fwd = kind == 0 || kind >= 3;
    GemmArgs a{};
    a.X = X;
    a.S_in = kind == 4 ? 0 : J;
    a.blocks = W;
    a.ptr = fwd ? dfp : dbp;
    a.idx = fwd ? dfi : dbi;
    a.order = tail > 0 ? (fwd ? dfo : dbo) : nullptr;
    a.tail = tail;
    a.bias = fwd ? bias : nullptr;
    a.pro_mode = pro;
    a.pro_scale = pro ? sc : nullptr;
    a.pro_shift = pro ? sh : nullptr;
    a.pro_F = F;
    a.spj_in = 1;
    a.alpha = 0.2f;
    a.Y = Y;
    a.S_out = J;
    a.addsrc = (fwd || std::getenv("LCN_DX_NORES")) ? nullptr : Y;
    a.epi_mode = kind >= 3 ? EPI_NONE : fwd ? EPI_BNFWD : EPI_BNBACK;
    a.stat = stat;
    a.epi_z = X2;
    a.epi_scale = sc;
    a.epi_shift = sh;
    a.epi_mean = mean;
    a.epi_rstd = rstd;
    a.epi_F = F;
    a.B = B;
    a.n_out_slabs = J;
    a.n_rt = (B + kRT - 1) / kRT;
    if (variant == 1) {
      a.pairs = fwd ? dfpp : dbpp;
      a.ment = fwd ? dfpm : dbpm;
      a.pair_order = tail > 0 ? (fwd ? dfpo : dbpo) : nullptr;
      a.n_pairs = (int)(fwd ? fpp : bpp).pairs.size();
    }
    a.n_blocks = nblk;
    return a;
  };
  GemmDwArgs d{};
  d.A = X;
  d.S_a = J;
  d.D = X2;
  d.S_d = J;
  d.spj_a = 1;
  d.spj_d = 1;
  d.alpha = 0.2f;
  d.d_z = X;
  d.d_scale = sc;
  d.d_shift = sh;
  d.d_c123 = c123;
  d.d_F = F;
  std::vector<int4> dw_map_host;
  std::vector<int4> grp;  // as lcn_api.cpp upload_dw_groups
  for (int so = 0; so < J; ++so) {
    std::vector<int> ids;
    for (int b = 0; b < nblk; ++b)
      if (blk[b].y == so) ids.push_back(b);
    for (size_t i = 0; i < ids.size(); i += 2)
      grp.push_back(make_int4(so, ids[i], i + 1 < ids.size() ? ids[i + 1] : -1, (int)(i / 2) | ((int)((ids.size() + 1) / 2) << 8)));
  }
  d.groups = dev(grp);
  d.ngroups = (int)grp.size();
  float* dzo;
  CK(hipMalloc(&dzo, (size_t)B * H * 4));
  d.dz_out = dzo;
  d.blk = dblk;
  d.nblk = nblk;
  d.B = B;
  {
    const int slots = std::getenv("LCN_DW_SLOTS") ? std::atoi(std::getenv("LCN_DW_SLOTS")) : gemm_dw_resident_slots();
    d.plan = make_dw_plan(B, (int)grp.size(), slots, nch, 128);
    if (std::getenv("LCN_DW_ITEM")) d.plan.item_rows = std::atoi(std::getenv("LCN_DW_ITEM"));
    if (std::getenv("LCN_DW_ROUNDS") && d.plan.stride == 8) d.plan.n_slots = 8 * d.plan.sub * std::atoi(std::getenv("LCN_DW_ROUNDS"));
    std::vector<int4> map = make_dw_wgmap((int)grp.size(), d.plan, B);
    if (std::getenv("LCN_DW_EQROUNDS") && d.plan.stride == 8) {  // experiment: rounds of equal size (batch segments)
      const int rounds = std::atoi(std::getenv("LCN_DW_EQROUNDS")), groups = (int)grp.size();
      const int n_items = (int)((B + d.plan.item_rows - 1) / d.plan.item_rows);
      d.plan.sub = 1;
      d.plan.n_slots = 8 * rounds;
      map.assign((size_t)8 * rounds * groups, make_int4(-1, 0, 0, 0));
      for (int x = 0; x < 8; ++x) {
        const int n = n_items > x ? (n_items - x + 7) / 8 : 0;
        for (int r = 0; r < rounds; ++r) {
          const int lo = (int)((int64_t)n * r / rounds), hi = (int)((int64_t)n * (r + 1) / rounds);
          for (int g = 0; g < groups; ++g)
            map[8 * ((size_t)r * groups + g) + x] = make_int4(g, 8 * r + x, x + 8 * lo, hi - lo);
        }
      }
    }
    dw_map_host = map;
    d.wgmap = dev(map);
    d.n_wg = (int)map.size();
    std::printf("dw plan: items of %d rows, stride %d, %d partials per block, %d workgroups (resident slots %d)\n",
                d.plan.item_rows, d.plan.stride, d.plan.n_slots, d.n_wg, slots);
  }
  d.part = part;
  // four blocks per workgroup (gemm_dw4.hip): the complete quads of every output slab
  GemmDwArgs d4 = d;
  int nblk4 = 0;
  {
    std::vector<int4> g4;
    for (int so = 0; so < J; ++so) {
      std::vector<int> ids;
      for (int b = 0; b < nblk; ++b)
        if (blk[b].y == so) ids.push_back(b);
      const int count = (int)ids.size() / 4;
      for (int q = 0; q < count; ++q) {
        g4.push_back(make_int4(so, 4, q, count));
        g4.push_back(make_int4(ids[4 * q], ids[4 * q + 1], ids[4 * q + 2], ids[4 * q + 3]));
        nblk4 += 4;
      }
    }
    d4.groups = dev(g4);
    d4.ngroups = (int)g4.size() / 2;
    const int slots4 = std::getenv("LCN_DW_SLOTS") ? std::atoi(std::getenv("LCN_DW_SLOTS")) : gemm_dw4_resident_slots();
    d4.plan = make_dw_plan(B, d4.ngroups, slots4, nch, 128);
    if (std::getenv("LCN_DW_ITEM")) d4.plan.item_rows = std::atoi(std::getenv("LCN_DW_ITEM"));
    const std::vector<int4> map4 = make_dw_wgmap(d4.ngroups, d4.plan, B);
    d4.wgmap = dev(map4);
    d4.n_wg = (int)map4.size();
    std::printf("dw4 plan: %d groups (%d of %d blocks), items of %d rows, stride %d, %d partials per block (sub %d), %d workgroups (resident slots %d)\n",
                d4.ngroups, nblk4, nblk, d4.plan.item_rows, d4.plan.stride, d4.plan.n_slots, d4.plan.sub, d4.n_wg, slots4);
  }

  struct Case { const char* name; int kind; int pro; int variant; };
  std::vector<Case> cases;
  const int nvar = argc > 4 ? std::atoi(argv[4]) : 1;
  for (int v = 0; v < nvar; ++v) {
    cases.push_back({"fwd raw +bnstat", 0, PRO_RAW, v});
    cases.push_back({"fwd bnact +bnstat", 0, PRO_BNACT, v});
    cases.push_back({"dx raw +bnback", 1, PRO_RAW, v});
    cases.push_back({"fwd raw no-epi", 3, PRO_RAW, v});
    cases.push_back({"fwd raw no-epi hotX", 4, PRO_RAW, v});
  }
  cases.push_back({"dw raw", 2, PRO_RAW, 0});
  cases.push_back({"dw bnact x bnback", 2, PRO_BNACT, 0});
  cases.push_back({"dw raw x bnback", 2, PRO_BNBACK, 0});
  cases.push_back({"dw4 raw", 5, PRO_RAW, 0});
  cases.push_back({"dw4 bnact x bnback", 5, PRO_BNACT, 0});
  cases.push_back({"dw4 raw x bnback", 5, PRO_BNBACK, 0});
  if (argc > 5) {  // keep only the cases whose name contains argv[5]
    std::vector<Case> keep;
    for (const Case& c : cases)
      if (std::strstr(c.name, argv[5])) keep.push_back(c);
    cases.swap(keep);
  }
  const int rounds = argc > 6 ? std::atoi(argv[6]) : 3;
  for (int r = 0; r < rounds; ++r) {
    for (const Case& c : cases) {
      auto run = [&]() {
        if (c.kind == 5) {
          d4.pro_scale = c.pro == PRO_BNACT ? sc : nullptr;
          d4.pro_shift = c.pro == PRO_BNACT ? sh : nullptr;
          d4.d_bnback = c.pro != PRO_RAW;
          launch_gemm_dw4(d4, s);  // (no reduce: the kernel alone)
        } else if (c.kind == 2) {
          d.pro_scale = c.pro == PRO_BNACT ? sc : nullptr;
          d.pro_shift = c.pro == PRO_BNACT ? sh : nullptr;
          d.d_bnback = c.pro != PRO_RAW;
          launch_gemm_dw(d, s);
          launch_dw_reduce(part, dw_plan_slots(d.plan), nblk, dblk, dW, H, H, H, s);
        } else {
          const GemmArgs ga = mk(c.kind, c.pro, c.variant);
          if (ga.pairs) launch_gemm_bs_pair(ga, s);
          else launch_gemm_bs(ga, s);
        }
      };
      run();
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int it = 0; it < iters; ++it) run();
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= iters;
      const double fl = c.kind == 5 ? flop * nblk4 / nblk : flop;
      std::printf("round %d v%d %-18s %8.1f us  %6.1f TFLOP/s  (%.1f%% of 157.3)\n", r, c.variant, c.name,
                  ms * 1e3, fl / (ms * 1e-3) / 1e12, 100.0 * fl / (ms * 1e-3) / 1e12 / 157.3);
    }
  }
#ifdef EXP_CLOCK
  for (int mode = 0; mode < 3; ++mode) {  // in-kernel clock and residency of the weight-gradient GEMM (raw; BN-backward D; + BN-apply A)
    const int grid = d.n_wg;
    uint64_t* clk;
    CK(hipMalloc(&clk, (size_t)grid * 32));
    d.clk = clk;
    d.pro_scale = mode == 2 ? sc : nullptr;
    d.pro_shift = mode == 2 ? sh : nullptr;
    d.d_bnback = mode >= 1;
    for (int it = 0; it < 1200; ++it) launch_gemm_dw(d, s);
    CK(hipStreamSynchronize(s));
    std::vector<uint64_t> st((size_t)4 * grid);
    CK(hipMemcpy(st.data(), clk, st.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> ghz, life;
    uint64_t t0 = ~0ull, t1 = 0;
    CK(hipMemset(clk, 0, (size_t)grid * 32));
    launch_gemm_dw(d, s);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(st.data(), clk, st.size() * 8, hipMemcpyDeviceToHost));
    for (int i = 0; i < grid; ++i) {
      if (st[4 * i + 3] == 0) continue;  // padding workgroups leave no stamps
      if (st[4 * i + 1] > 100) ghz.push_back((double)st[4 * i] / (double)st[4 * i + 1] * 0.1);
      life.push_back((double)st[4 * i + 1] * 0.01);
      t0 = std::min(t0, st[4 * i + 2]);
      t1 = std::max(t1, st[4 * i + 3]);
    }
    std::sort(ghz.begin(), ghz.end());
    std::sort(life.begin(), life.end());
    std::printf("dw mode %d: in-kernel clock (GHz) min %.3f median %.3f max %.3f; launch span %.1f us; workgroup life (us) min %.1f median %.1f max %.1f; resident per 5%% bin:",
                mode, ghz.front(), ghz[ghz.size() / 2], ghz.back(), (double)(t1 - t0) * 0.01, life.front(),
                life[life.size() / 2], life.back());
    const double span = (double)(t1 - t0);
    std::vector<double> act(20, 0.0);
    for (int i = 0; i < grid; ++i) {
      if (st[4 * i + 3] == 0) continue;
      const double b0 = (st[4 * i + 2] - t0) / span * 20, b1 = (st[4 * i + 3] - t0) / span * 20;
      for (int b = (int)b0; b < 20 && b <= (int)b1; ++b)
        act[b] += std::min(b1, (double)b + 1) - std::max(b0, (double)b);
    }
    for (double v : act) std::printf(" %.0f", v);
    {  // median life by kind of slot: XCD-affine (j < 8) / dealt (j >= 8) two-block, one-block; and by XCD
      std::vector<double> cat[3], byx[8];
      for (int i = 0; i < grid; ++i) {
        if (st[4 * i + 3] == 0 || dw_map_host[i].x < 0) continue;
        const double l = (double)st[4 * i + 1] * 0.01;
        const bool two = grp[dw_map_host[i].x].z >= 0;
        cat[!two ? 2 : dw_map_host[i].y < 8 ? 0 : 1].push_back(l);  // first round / later rounds / one-block
        if (two) byx[i & 7].push_back(l);
      }
      std::printf("; median life affine/dealt/one-block:");
      for (auto& c : cat) { std::sort(c.begin(), c.end()); std::printf(" %.0f", c.empty() ? 0.0 : c[c.size() / 2]); }
      std::printf("; by XCD:");
      for (auto& c : byx) { std::sort(c.begin(), c.end()); std::printf(" %.0f", c.empty() ? 0.0 : c[c.size() / 2]); }
    }
    std::printf("; life deciles:");
    for (int q = 0; q <= 10; ++q) std::printf(" %.0f", life[std::min(life.size() - 1, life.size() * q / 10)]);
    std::printf("\n");
    d.clk = nullptr;
    CK(hipFree(clk));
  }
  {  // in-kernel clock of the no-epilogue forward GEMM after sustained load,
     // and the occupancy profile of its last launch (how long the tail is)
    GemmArgs a = mk(3, PRO_RAW, 0);
    const int grid = 8 * (((a.n_rt + kGemmWaves - 1) / kGemmWaves + 7) / 8) * a.n_out_slabs;
    for (int it = 0; it < 1500; ++it) launch_gemm_bs(a, s);   // > 1 s of back-to-back launches
    CK(hipStreamSynchronize(s));
    std::vector<uint64_t> st((size_t)4 * grid);
    CK(hipMemcpy(st.data(), stat, st.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> ghz;
    uint64_t t0 = ~0ull, t1 = 0;
    for (int i = 0; i < grid; ++i) {
      if (st[4 * i + 1] > 100) ghz.push_back((double)st[4 * i] / (double)st[4 * i + 1] * 0.1);
      t0 = std::min(t0, st[4 * i + 2]);
      t1 = std::max(t1, st[4 * i + 3]);
    }
    std::sort(ghz.begin(), ghz.end());
    std::printf("in-kernel clock (GHz) over %zu workgroups: min %.3f median %.3f max %.3f\n", ghz.size(),
                ghz.front(), ghz[ghz.size() / 2], ghz.back());
    // resident workgroups over time, in 20 bins of the launch
    const double span = (double)(t1 - t0);
    std::vector<double> act(20, 0.0);
    double wsum = 0;
    for (int i = 0; i < grid; ++i) {
      const double b0 = (st[4 * i + 2] - t0) / span * 20, b1 = (st[4 * i + 3] - t0) / span * 20;
      wsum += (double)(st[4 * i + 3] - st[4 * i + 2]);
      for (int b = (int)b0; b < 20 && b <= (int)b1; ++b)
        act[b] += std::min(b1, (double)b + 1) - std::max(b0, (double)b);
    }
    std::printf("launch span %.1f us, mean workgroup life %.1f us; resident workgroups per 5%% bin:", span * 0.01,
                wsum / grid * 0.01);
    for (double v : act) std::printf(" %.0f", v);
    std::printf("\n");
  }
#endif
  CK(hipGetLastError());
  return 0;
}
