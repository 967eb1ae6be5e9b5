// Host AddressSanitizer driver for the C ABI (host ASan on the shim).
//
// Built by `make -C unet-embroidery-seg_amd/csrc asan` from the library's own sources compiled
// host-only (hipcc --offload-host-only -fsanitize=address: no device code, nothing is launched) and
// run by tests/test_cabi_asan.py on the CPU.  It drives every host-side code path of the ABI that
// runs before a launch:
//   1. the shape-driven host logic -- kernel-configuration queries, tile / workspace / partial-buffer
//      geometry, the fused-dgrad row count, the pack-tile count -- over a grid of shapes that covers
//      every layer of the BASELINE models plus ragged and degenerate ones (results are written into
//      exactly-sized arrays, so an out-of-bounds write is an ASan report);
//   2. the argument checks of the launching entry points: each call below must be refused with
//      status 1 and a message, before any HIP call;
//   3. the augmentation's descriptor / table validation, which walks caller-provided host tables: a
//      valid first sample (its tables walked to the last entry, in exactly-sized heap arrays) followed
//      by a second sample that breaks one rule per case.
// Exit status 0 = every expectation held (and ASan found nothing: it aborts the process otherwise).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/unetseg_hip.h"

static int g_fail = 0, g_checks = 0;

#define EXPECT(cond, ...)                    \
  do {                                       \
    ++g_checks;                              \
    if (!(cond)) {                           \
      ++g_fail;                              \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);     \
      std::fprintf(stderr, "\n");            \
    }                                        \
  } while (0)

// a refused call: status 1 and a non-empty message naming the entry point
static void refused(int rc, const char* what) {
  const char* e = unetseg_last_error();
  EXPECT(rc == 1 && e && e[0], "%s: rc=%d err='%s' (expected an argument error)", what, rc, e ? e : "");
}

// never dereferenced on the host: the argument checks fail first
static void* const D = reinterpret_cast<void*>(static_cast<uintptr_t>(4096));
static float* const DF = reinterpret_cast<float*>(static_cast<uintptr_t>(4096));

static void shape_queries() {
  const int Ns[] = {1, 2, 3, 8, 16};
  const int Hs[] = {1, 7, 8, 15, 16, 17, 32, 33, 64, 128, 256, 512};
  const int Cs[] = {3, 8, 32, 40, 64, 128, 192, 256, 512, 1024, 2048, 3072};
  const int Ks[] = {1, 2, 32, 64, 128, 256, 512, 2048};
  long long sink = 0;
  for (int dt = 0; dt < 2; ++dt)
    for (int n : Ns)
      for (int h : Hs)
        for (int c : Cs)
          for (int k : Ks)
            for (int r = 1; r <= 3; r += 2)
              for (int st = 1; st <= 2; ++st) {
                const int pad = r / 2;
                const int p = (h + 2 * pad - r) / st + 1;
                int taps = -7;
                sink += unetseg_conv2d_fwd_config(dt, c, c, 0, 0, n, h, h, k, r, r, st, pad, &taps);
                sink += taps;
                // virtual concat: two sources, the second at a wider pixel stride
                sink += unetseg_conv2d_fwd_config(dt, c, c, 64, 128, n, h, h, k, r, r, st, pad, &taps);
                sink += unetseg_conv2d_fwd_tile_m(dt, c, c, 0, 0, n, h, h, k, r, r, st, pad);
                int cfg[4], tp[4];
                const int ncls = unetseg_conv2d_dgrad_config(dt, k, n, p, p, k, c, r, r, st, pad, c, h, h, cfg, tp);
                EXPECT(ncls >= 0 && ncls <= st * st, "dgrad_config classes %d", ncls);
                sink += ncls;
                int sp = -1;
                sink += unetseg_conv2d_wgrad_config(dt, c, c, 0, 0, n, h, h, k, k, r, r, st, pad, &sp);
                sink += sp;
                sink += (long long)unetseg_conv2d_wgrad_workspace(dt, n, p, p, k, c, r, r);
                for (int post = 1; post <= 2; ++post)
                  sink += unetseg_conv2d_dgrad_post(dt, nullptr, k, n, p, p, nullptr, k, c, r, r, st, pad, nullptr, c,
                                                    h, h, post, nullptr, c, nullptr, nullptr, nullptr, nullptr,
                                                    nullptr, 0, nullptr);
                if (r == 1 && st == 1) {
                  sink += unetseg_conv2d_fwd_bnrelu_in_config(dt, c, c, n, h, h, k);
                  sink += unetseg_pack_tiles(k, c, 1);
                } else {
                  sink += unetseg_pack_tiles(k, c, r * r);
                }
              }
  for (int n : Ns)
    for (int h : Hs) {
      int sp = -1;
      sink += unetseg_stem_config(n, h, h, 64, &sp) + sp;
      sink += unetseg_stem_fwd_tile_m(n, h, h, 64);
      sink += (long long)unetseg_stem_wgrad_workspace(n, h, h, 64);
      for (int k = 1; k <= 2; ++k) sink += unetseg_conv2d_fwd_head_ok(1, 64, n, h, h, 64, k);
      for (int c : Cs) {
        const long M = (long)n * h * h;
        for (int dt = 0; dt < 2; ++dt) {
          int tv = -1, ppb = -1;
          sink += unetseg_reduce_tiles(dt, M, c, &tv, &ppb) + tv + ppb;
          sink += unetseg_upsample2x_bwd_tiles(dt, n, h, h, c);
        }
        sink += unetseg_channel_stats_tiles(M, 256);
      }
      const long M = (long)n * h * h;
      sink += unetseg_pw_small_tile(M) + unetseg_pw_small_tiles(M) + unetseg_attn_bwd1_tiles(M) +
              unetseg_pw_head_tiles(M);
      sink += (long long)unetseg_lovasz_workspace(n, (long)h * h);
      sink += (long long)unetseg_bce_workspace(n, (long)h * h);
      sink += (long long)unetseg_masked_loss_workspace(n, (long)h * h);
      for (int c = 2; c <= 32; c += 10) sink += (long long)unetseg_mc_loss_workspace(n, c, (long)h * h);
    }
  for (long long nw = 1; nw <= 600; nw += 53)
    for (long long nh = 1; nh <= 600; nh += 61) sink += unetseg_augment_tables_len(nw, nh, 6, 9, nw & 1);
  EXPECT(sink != 0x7fffffffffffffffLL, "sink");
  // identity
  EXPECT(unetseg_abi_version() == 1, "abi version");
  EXPECT(unetseg_conv_tile_m() > 0, "conv tile");
}

static void argument_checks() {
  // convolution
  refused(unetseg_conv2d_fwd(7, D, 64, 64, nullptr, 0, 0, 1, 8, 8, D, 64, 3, 3, 1, 1, nullptr, 0, D, 64, nullptr,
                             nullptr), "conv2d_fwd bad dtype");
  refused(unetseg_conv2d_fwd(1, nullptr, 64, 64, nullptr, 0, 0, 1, 8, 8, D, 64, 3, 3, 1, 1, nullptr, 0, D, 64,
                             nullptr, nullptr), "conv2d_fwd null x");
  refused(unetseg_conv2d_fwd(1, D, 64, 32, nullptr, 0, 0, 1, 8, 8, D, 64, 3, 3, 1, 1, nullptr, 0, D, 64, nullptr,
                             nullptr), "conv2d_fwd ld < c");
  refused(unetseg_conv2d_fwd(1, D, 64, 64, nullptr, 0, 0, -1, 8, 8, D, 64, 3, 3, 1, 1, nullptr, 0, D, 64, nullptr,
                             nullptr), "conv2d_fwd negative batch");
  refused(unetseg_conv2d_fwd_bnrelu_in(1, D, 64, 64, 1, 8, 8, D, 64, nullptr, nullptr, nullptr, 0, D, 64, nullptr,
                                       nullptr), "fwd_bnrelu_in no coefficients");
  refused(unetseg_conv2d_fwd_head(1, D, 64, 1, 8, 8, D, DF, D, 64, 3, DF, DF, DF, nullptr), "fwd_head k=3");
  refused(unetseg_conv2d_dgrad(1, nullptr, 64, 1, 8, 8, D, 64, 64, 3, 3, 1, 1, D, 64, 8, 8, 0, nullptr),
          "dgrad null dy");
  refused(unetseg_conv2d_dgrad(3, D, 64, 1, 8, 8, D, 64, 64, 3, 3, 1, 1, D, 64, 8, 8, 0, nullptr), "dgrad dtype");
  refused(unetseg_conv2d_dgrad_post(1, D, 64, 1, 8, 8, D, 64, 64, 3, 3, 1, 1, D, 64, 8, 8, 3, D, 64, DF, DF, DF, DF,
                                    DF, 1, nullptr), "dgrad_post post=3");
  {
    const int rows = unetseg_conv2d_dgrad_post(1, nullptr, 64, 2, 32, 32, nullptr, 64, 64, 3, 3, 1, 1, nullptr, 64,
                                               32, 32, 2, nullptr, 64, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                                               nullptr);
    EXPECT(rows > 0, "dgrad_post rows query %d", rows);
    refused(unetseg_conv2d_dgrad_post(1, D, 64, 2, 32, 32, D, 64, 64, 3, 3, 1, 1, D, 64, 32, 32, 2, D, 64, DF, DF,
                                      DF, DF, DF, rows + 1, nullptr), "dgrad_post wrong rows");
    refused(unetseg_conv2d_dgrad_post(1, D, 64, 2, 32, 32, D, 64, 64, 3, 3, 1, 1, D, 64, 32, 32, 2, D, 64, nullptr,
                                      DF, DF, DF, DF, rows, nullptr), "dgrad_post BN without coefficients");
  }
  refused(unetseg_conv2d_wgrad(1, D, 64, 64, nullptr, 0, 0, 1, 8, 8, D, 64, 64, 3, 3, 1, 1, DF, 0, nullptr, 64, 0,
                               nullptr), "wgrad null dw");
  refused(unetseg_conv2d_wgrad(1, D, 64, 64, nullptr, 0, 0, 16, 128, 128, D, 64, 64, 3, 3, 1, 1, DF, 1, DF, 64, 0,
                               nullptr), "wgrad workspace too small");
  refused(unetseg_conv2d_wgrad_bnrelu_in(1, D, 64, 64, 1, 8, 8, D, 64, 64, nullptr, nullptr, DF, 1 << 20, DF, 64, 0,
                                         nullptr), "wgrad_bnrelu_in no coefficients");
  refused(unetseg_conv2d_fwd_affine(1, D, 64, 64, nullptr, 0, 0, 1, 8, 8, D, 64, 3, 3, 1, 1, nullptr, DF, 1, D, 64,
                                    nullptr), "fwd_affine no scale");
  refused(unetseg_pack_conv_weight(1, nullptr, 64, 64, 3, 3, 64, D, D, nullptr), "pack null w");
  refused(unetseg_pack_conv_weight(1, DF, 64, 64, 3, 3, 32, D, D, nullptr), "pack cpad < c");
  refused(unetseg_pack_conv_weights(1, nullptr, 3, 10, nullptr), "pack_conv_weights null desc");
  refused(unetseg_stem_fwd(nullptr, 1, 64, 64, D, 64, D, 64, DF, nullptr), "stem_fwd null x");
  refused(unetseg_stem_wgrad(D, 1, 64, 64, D, 64, 64, DF, 1, DF, 3, 0, nullptr), "stem_wgrad workspace");
  refused(unetseg_pack_input(1, nullptr, 1, 3, 8, 8, 8, D, nullptr), "pack_input null");
  refused(unetseg_pack_input(1, DF, 1, 9, 8, 8, 8, D, nullptr), "pack_input c > cpad");
  // BatchNorm
  refused(unetseg_bn_finalize(nullptr, 64, 4, 512, 128, DF, DF, DF, DF, nullptr, 0.1f, 1e-5f, DF, DF, DF, DF, nullptr),
          "bn_finalize null part");
  refused(unetseg_bn_apply(1, D, 64, DF, DF, nullptr, 0, nullptr, nullptr, 7, 1, D, 64, 64, 64, nullptr),
          "bn_apply res_mode");
  refused(unetseg_bn_apply(1, D, 64, DF, DF, nullptr, 0, nullptr, nullptr, 1, 1, D, 64, 64, 64, nullptr),
          "bn_apply res_mode 1 without residual");
  refused(unetseg_bn_apply_mask(1, D, 64, DF, DF, D, 64, nullptr, nullptr, 1, D, 64, 64, 64, nullptr, nullptr),
          "bn_apply_mask null mask");
  refused(unetseg_bn_bwd_reduce(1, D, 64, nullptr, 64, nullptr, nullptr, D, 64, DF, DF, nullptr, 0, nullptr, nullptr,
                                64, 64, nullptr, 1, nullptr), "bn_bwd_reduce null part");
  refused(unetseg_bn_bwd_finalize(DF, 64, 1, 64, 3, DF, DF, DF, DF, nullptr, nullptr, nullptr, nullptr, DF, nullptr),
          "bn_bwd_finalize nbranch=3");
  refused(unetseg_channel_stats(1, D, 64, 100, 64, 0, DF, nullptr), "channel_stats tile 0");
  // pooling / resampling
  refused(unetseg_maxpool_fwd(1, D, 64, 1, 8, 8, 64, 0, 2, 0, D, 64, nullptr, nullptr, nullptr, nullptr),
          "maxpool k=0");
  refused(unetseg_upsample2x_fwd(1, nullptr, 64, 1, 8, 8, 64, 1, D, 64, nullptr), "upsample null x");
  refused(unetseg_upsample2x_bwd_relu(1, D, 64, 1, 8, 8, 64, 1, D, 64, D, 64, DF, 99999, nullptr),
          "upsample_bwd_relu rows");
  refused(unetseg_resize_bilinear_fwd(1, D, 64, 1, 8, 8, 64, 0, 16, 0, D, 64, nullptr), "resize oh=0");
  refused(unetseg_pad2d_fwd(1, D, 64, 1, 8, 8, 64, 4, 4, 9, 9, D, 64, nullptr), "pad overhang");
  // heads, attention gate
  refused(unetseg_pw_small_fwd(1, D, 64, 100, 100, 64, 3, DF, DF, DF, nullptr, nullptr), "pw_small k=3");
  refused(unetseg_pw_small_fwd(1, D, 64, 100, 100, 64, 2, DF, DF, DF, DF, nullptr), "pw_small stats with k=2");
  refused(unetseg_pw_small_bwd_relu(0, DF, D, 64, 100, 100, 64, 1, DF, D, 64, DF, DF, DF, nullptr),
          "pw_small_bwd_relu fp32");
  refused(unetseg_attn_bwd1(1, D, 48, D, 48, DF, DF, DF, DF, D, 48, 0, DF, 100, 48, DF, nullptr),
          "attn_bwd1 C/V not a power of two");
  refused(unetseg_pw_head_fwd(1, D, 64, 100, 100, 64, 33, DF, DF, DF, nullptr), "pw_head k=33");
  // losses, metrics, optimizer
  refused(unetseg_lovasz_fwd(DF, 2, nullptr, 2, 100, D, 1 << 20, DF, DF, nullptr), "lovasz null targets");
  refused(unetseg_lovasz_fwd(DF, 2, reinterpret_cast<const int64_t*>(D), 2, 100, D, 1, DF, DF, nullptr),
          "lovasz workspace");
  refused(unetseg_bce_fwd(DF, 3, reinterpret_cast<const int64_t*>(D), 2, 100, nullptr, D, 1 << 20, DF, DF, nullptr),
          "bce nch=3");
  refused(unetseg_masked_loss_fwd(DF, 2, reinterpret_cast<const int64_t*>(D), 2, 100, 255, 5, nullptr, D, 1 << 20,
                                  DF, DF, nullptr), "masked loss kind");
  refused(unetseg_mc_loss_fwd(DF, reinterpret_cast<const int64_t*>(D), 2, 40, 100, nullptr, 40, 0, -1.f, 0.f,
                              nullptr, 0, 1.f, 1e-5f, D, 1 << 20, DF, nullptr), "mc_loss C=40");
  refused(unetseg_softmax_resize_argmax(DF, 2, 8, 8, 0, 0, 9, 8, 16, 16, reinterpret_cast<int32_t*>(D), nullptr),
          "softmax_resize crop outside");
  refused(unetseg_adam(nullptr, DF, DF, DF, 10, 1e-3f, 0.9f, 0.999f, 1e-8f, 0.f, 1, nullptr, nullptr), "adam null p");
  refused(unetseg_adam(DF, DF, DF, DF, 10, 1e-3f, 0.9f, 0.999f, 1e-8f, 0.f, 0, nullptr, nullptr), "adam step 0");
  refused(unetseg_linear_fwd(nullptr, DF, DF, 2, 8, 8, 0, 0.f, 0, nullptr, nullptr, nullptr, DF, nullptr),
          "linear_fwd null x");
  refused(unetseg_ce_fwd(DF, reinterpret_cast<const int64_t*>(D), 0, 3, DF, DF, nullptr), "ce B=0");
}

// ---- augmentation descriptors / tables ----------------------------------------------------------
enum { D_SRC, D_MSK, D_TMP, D_RSZ, D_IW, D_IH, D_NW, D_NH, D_DX, D_DY, D_FLIP, D_Y0, D_ROWS, D_KSH, D_KSV, D_TAB,
       D_HSV, D_MIW, D_MIH, AUG_DESC = 20 };

struct Sample {
  long long iw, ih, nw, nh, miw, mih, ksh, ksv, hsv;
};

// one sample's tables in the layout pack_batch writes (utils/hf_dataloader.py): horizontal windows
// [nw][2] + taps [nw][ksh], vertical [nh][2] + [nh][ksv], nearest x [nw], nearest y [nh], LUTs
static void append_tables(const Sample& s, std::vector<int>& t) {
  for (long long x = 0; x < s.nw; ++x) {
    const long long x0 = x * s.iw / s.nw;
    const long long cnt = (x0 + s.ksh <= s.iw) ? s.ksh : s.iw - x0;
    t.push_back((int)x0);
    t.push_back((int)cnt);
  }
  for (long long i = 0; i < s.nw * s.ksh; ++i) t.push_back(1 << 20);
  for (long long y = 0; y < s.nh; ++y) {
    const long long y0 = y * s.ih / s.nh;
    const long long cnt = (y0 + s.ksv <= s.ih) ? s.ksv : s.ih - y0;
    t.push_back((int)y0);
    t.push_back((int)cnt);
  }
  for (long long i = 0; i < s.nh * s.ksv; ++i) t.push_back(1 << 20);
  for (long long x = 0; x < s.nw; ++x) t.push_back((int)(x * s.miw / s.nw));
  for (long long y = 0; y < s.nh; ++y) t.push_back((int)(y * s.mih / s.nh));
  const long long used = 2 * s.nw + s.nw * s.ksh + 2 * s.nh + s.nh * s.ksv + s.nw + s.nh;
  const long long len = unetseg_augment_tables_len(s.nw, s.nh, s.ksh, s.ksv, s.hsv);
  for (long long i = used; i < len; ++i) t.push_back(i & 255);
}

static void augment_checks() {
  const Sample good{40, 30, 52, 37, 40, 30, 6, 9, 1};
  const Sample second{25, 20, 17, 11, 25, 20, 4, 4, 0};
  enum Break { NONE, EMPTY, ROWS, SRC, MSK, TMP, RSZ, TAB, HWIN, HCNT, NX, VWIN, NY, NCASE };
  for (int b = NONE; b < NCASE; ++b) {
    std::vector<int> tab;
    append_tables(good, tab);
    const long long tab1 = (long long)tab.size();
    append_tables(second, tab);
    std::vector<long long> desc(2 * AUG_DESC, 0);
    long long src = 0, msk = 0, tmp = 0, rsz = 0;
    const Sample* ss[2] = {&good, &second};
    for (int i = 0; i < 2; ++i) {
      long long* d = desc.data() + i * AUG_DESC;
      const Sample& s = *ss[i];
      d[D_SRC] = src; d[D_MSK] = msk; d[D_TMP] = tmp; d[D_RSZ] = rsz;
      d[D_IW] = s.iw; d[D_IH] = s.ih; d[D_NW] = s.nw; d[D_NH] = s.nh; d[D_KSH] = s.ksh; d[D_KSV] = s.ksv;
      d[D_Y0] = 0; d[D_ROWS] = s.ih; d[D_TAB] = i ? tab1 : 0; d[D_HSV] = s.hsv; d[D_MIW] = s.miw; d[D_MIH] = s.mih;
      src += s.iw * s.ih * 3; msk += s.miw * s.mih; tmp += s.ih * s.nw * 3; rsz += s.nh * s.nw * 3;
    }
    long long* d1 = desc.data() + AUG_DESC;
    long long src_bytes = src, n_tab = (long long)tab.size();
    const long long b1 = tab1;                                           // sample 1's tables
    const long long v1 = b1 + 2 * second.nw + second.nw * second.ksh;   // its vertical windows
    const long long nx1 = v1 + 2 * second.nh + second.nh * second.ksv;  // its nearest-x table
    switch (b) {
      case EMPTY: d1[D_NW] = 0; break;
      case ROWS: d1[D_ROWS] = second.ih + 1; break;
      case SRC: src_bytes -= 1; break;
      case MSK: d1[D_MSK] += 1; break;
      case TMP: d1[D_TMP] = tmp; break;
      case RSZ: d1[D_RSZ] = -1; break;
      case TAB: n_tab -= 1; break;
      case HWIN: tab[b1 + 2 * (second.nw - 1)] = (int)second.iw; break;
      case HCNT: tab[b1 + 1] = (int)second.ksh + 1; break;
      case NX: tab[nx1 + second.nw - 1] = (int)second.miw; break;
      case VWIN: tab[v1] = -1; break;
      case NY: tab[nx1 + second.nw + second.nh - 1] = -3; break;
      default: break;
    }
    if (b == NONE) continue;  // a valid batch would go on to launch (no device here)
    // exactly-sized host copies: a read past the end of either is an ASan report
    std::vector<long long> dh(desc);
    std::vector<int> th(tab.begin(), tab.begin() + (b == TAB ? n_tab : (long long)tab.size()));
    const int rc = unetseg_augment_batch(dh.data(), reinterpret_cast<const long long*>(D), 2, th.data(),
                                         reinterpret_cast<const int*>(D), n_tab, reinterpret_cast<const uint8_t*>(D),
                                         src_bytes, reinterpret_cast<const uint8_t*>(D), msk,
                                         reinterpret_cast<uint8_t*>(D), tmp, reinterpret_cast<uint8_t*>(D), rsz, 32,
                                         32, 2, 1, DF, reinterpret_cast<long long*>(D), nullptr, nullptr);
    refused(rc, "augment_batch broken sample");
    EXPECT(std::strstr(unetseg_last_error(), "sample 1") != nullptr, "augment case %d: '%s'", b, unetseg_last_error());
  }
  refused(unetseg_augment_batch(nullptr, nullptr, 1, nullptr, nullptr, 0, nullptr, 0, nullptr, 0, nullptr, 0, nullptr,
                                0, 8, 8, 2, 1, nullptr, nullptr, nullptr, nullptr), "augment_batch null");
}

int main() {
  shape_queries();
  argument_checks();
  augment_checks();
  std::printf("cabi_asan: %d checks, %d failed\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
