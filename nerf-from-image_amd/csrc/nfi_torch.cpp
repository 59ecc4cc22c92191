// TORCH_LIBRARY(nfi, ...) operators over the nfi C-ABI (include/nfi.h): the drop-in boundary of
// SURVEY §8(b) for callers that go through the PyTorch dispatcher — TorchScript (the reference's
// lib/nerf_utils.py functions are @torch.jit.script) and the C++ frontend — instead of the ctypes
// binding (nfi/_lib.py).  One implementation: every op launches the same HIP kernels through the
// C-ABI on the current HIP stream of its tensors' device; no CPU path (a CPU tensor raises).
//
//   nfi::rays(cam, focal?, center?, bbox?, H, W, scene_range) -> (ro, rd, near, far)
//       get_ray_bundle + F.normalize + compute_near_far_planes (run.py:193-200); autograd to cam, focal
//   nfi::pack_decoder(w1, b1, w2, b2, attention_values=-1) -> dec   EqualizedLinear gains folded (stylegan.py:173-176)
//   nfi::volume_render(planes_tm, palette?, ro, rd, near, far, dec, samples, fine, white_background,
//                      randomize, scene_range, inv_alpha, beta, heads, seed, u_coarse?, u_fine?)
//       -> (rgb, depth, mask)                         run.py:202-348 fused; autograd to planes_tm,
//                                                     palette, ro, rd
//   nfi::volume_render_fwd / nfi::volume_render_bwd   its two halves as plain ops (CUDA + Meta kernels)
//   nfi::sample_pdf, nfi::compute_near_far_planes, nfi::cumprod_exclusive,
//   nfi::render_volume_density_weights_only           the nerf_utils seams (nerf_utils.py:20-25,
//                                                     166-182, 185-224, 227-275)
//   nfi::render_fwd / nfi::render_bwd                 SURVEY §8(b)'s names on the reference layouts
//                                                     (channel-major planes, gain-scaled W1s/W2s)
//   nfi::composite_fwd/_bwd, nfi::triplane_mlp_fwd/_bwd  per-stage ops (nerf_utils.py:125-163;
//                                                     generator.py:587-681)
#include <cstring>
#include <cstdlib>
#include <cmath>
#include <string>
#include <vector>

#include <c10/hip/HIPStream.h>
#include <torch/autograd.h>
#include <torch/library.h>
#include <torch/torch.h>

#include "../../include/nfi.h"

namespace {

using torch::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

void check(int32_t rc, const char* what) {
  TORCH_CHECK(rc == 0, "nfi: ", what, " failed (", rc, "): ", nfi_last_error());
}

void* stream_of(const Tensor& t) { return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void require(const Tensor& t, const char* name) {
  TORCH_CHECK(t.defined(), "nfi: ", name, " is undefined");
  TORCH_CHECK(t.is_cuda(), "nfi ops run on HIP devices only (", name, " is on ", t.device(), ")");
  TORCH_CHECK(t.scalar_type() == torch::kFloat, "nfi ops need float32 tensors (", name, " is ", t.scalar_type(), ")");
}

const float* fptr(const c10::optional<Tensor>& t) { return (t && t->defined()) ? t->data_ptr<float>() : nullptr; }
float* mptr(const Tensor& t) { return t.defined() ? t.data_ptr<float>() : nullptr; }

nfi_camera camera(const Tensor& cam, const c10::optional<Tensor>& focal, const c10::optional<Tensor>& center,
                  const c10::optional<Tensor>& bbox, int64_t H, int64_t W) {
  nfi_camera c{};
  c.cam = cam.data_ptr<float>();
  c.focal = fptr(focal);
  c.center = fptr(center);
  c.bbox = fptr(bbox);
  c.B = (int32_t)cam.size(0);
  c.H = (int32_t)H;
  c.W = (int32_t)W;
  return c;
}

// ---- rays --------------------------------------------------------------------------------------
struct RaysFn : public torch::autograd::Function<RaysFn> {
  static variable_list forward(AutogradContext* ctx, Tensor cam, Tensor focal, c10::optional<Tensor> center,
                               c10::optional<Tensor> bbox, int64_t H, int64_t W, double scene_range) {
    require(cam, "cam");
    const c10::DeviceGuard guard(cam.device());
    const int64_t B = cam.size(0), n = B * H * W;
    Tensor cam_c = cam.contiguous();
    Tensor foc_c = focal.defined() ? focal.contiguous() : Tensor();
    c10::optional<Tensor> cen_c = center ? c10::optional<Tensor>(center->contiguous()) : c10::nullopt;
    c10::optional<Tensor> bb_c = bbox ? c10::optional<Tensor>(bbox->contiguous()) : c10::nullopt;
    auto o = cam.options();
    Tensor ro = torch::empty({B, H, W, 3}, o), rd = torch::empty({B, H, W, 3}, o);
    Tensor nr = torch::empty({B, H, W}, o), fr = torch::empty({B, H, W}, o);
    Tensor ws = torch::empty({2 + n}, o.dtype(torch::kInt32));
    nfi_camera c = camera(cam_c, foc_c.defined() ? c10::optional<Tensor>(foc_c) : c10::nullopt, cen_c, bb_c, H, W);
    check(nfi_rays_forward(&c, (float)scene_range, ro.data_ptr<float>(), rd.data_ptr<float>(), nr.data_ptr<float>(),
                           fr.data_ptr<float>(), (uint32_t*)ws.data_ptr<int32_t>(), stream_of(cam)),
          "nfi_rays_forward");
    ctx->save_for_backward({cam_c, foc_c, cen_c ? *cen_c : Tensor(), bb_c ? *bb_c : Tensor()});
    ctx->saved_data["H"] = H;
    ctx->saved_data["W"] = W;
    ctx->mark_non_differentiable({nr, fr});
    return {ro, rd, nr, fr};
  }

  static variable_list backward(AutogradContext* ctx, variable_list g) {
    auto s = ctx->get_saved_variables();
    const Tensor cam = s[0], focal = s[1], center = s[2], bbox = s[3];
    const int64_t H = ctx->saved_data["H"].toInt(), W = ctx->saved_data["W"].toInt();
    const int64_t B = cam.size(0), n = B * H * W;
    auto o = cam.options();
    Tensor g_ro = g[0].defined() ? g[0].contiguous() : torch::zeros({n, 3}, o);
    Tensor g_rd = g[1].defined() ? g[1].contiguous() : torch::zeros({n, 3}, o);
    Tensor contrib = torch::empty({n, 16}, o);
    auto opt = [](const Tensor& t) { return t.defined() ? c10::optional<Tensor>(t) : c10::nullopt; };
    nfi_camera c = camera(cam, opt(focal), opt(center), opt(bbox), H, W);
    void* st = stream_of(cam);
    check(nfi_rays_backward(&c, g_ro.data_ptr<float>(), g_rd.data_ptr<float>(), contrib.data_ptr<float>(), st),
          "nfi_rays_backward");
    Tensor red = torch::empty({B, 16}, o), ws = torch::empty({B * 64 * 16}, o);
    check(nfi_segment_sum(contrib.data_ptr<float>(), (int32_t)B, (int32_t)(H * W), 16, red.data_ptr<float>(),
                          ws.data_ptr<float>(), st),
          "nfi_segment_sum");
    Tensor d_cam = torch::zeros({B, 4, 4}, o);
    d_cam.slice(1, 0, 3).copy_(red.slice(1, 0, 12).view({B, 3, 4}));
    d_cam.select(1, 3).select(1, 3).copy_(red.select(1, 12));
    Tensor d_focal = focal.defined() ? red.select(1, 13).clone() : Tensor();
    return {d_cam, d_focal, Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

std::tuple<Tensor, Tensor, Tensor, Tensor> rays(const Tensor& cam, const c10::optional<Tensor>& focal,
                                                const c10::optional<Tensor>& center,
                                                const c10::optional<Tensor>& bbox, int64_t H, int64_t W,
                                                double scene_range) {
  auto r = RaysFn::apply(cam, focal ? *focal : Tensor(), center, bbox, H, W, scene_range);
  return {r[0], r[1], r[2], r[3]};
}

// ---- decoder -------------------------------------------------------------------------------------
// scaled false: the EqualizedLinear gains 1/sqrt(fan_in) are folded here; true: weights already scaled
// (W1s, W2s).  attention_values: 0 = the wide-sigmoid colour head (w2 [4,64]: distance + 3 features,
// zero-padded to the kernels' 11 rows: rows the head never reads); 1..10 = the attention head with
// that many logits (w2 [N+1,64]): for N < 10 the missing logits get zero weights and a -1e30 bias, so
// their softmax terms exp(-1e30 - max) are exactly 0 and the head is the N-value one (render.py
// attention_padded does the same; a ZERO-biased padded logit would put exp(-max) of mass on palette
// rows N..9); -1 = inferred from the rows: 11 -> 10 attention values, 4 -> the colour head, 33 -> the
// view-direction decoder; any other row count needs attention_values.
Tensor pack_with_gains(const Tensor& w1, const Tensor& b1, const Tensor& w2_in, const Tensor& b2_in, bool scaled,
                       int64_t attention_values) {
  require(w1, "w1");
  require(b1, "b1");
  require(w2_in, "w2");
  require(b2_in, "b2");
  TORCH_CHECK(w1.dim() == 2 && w1.size(0) == 64 && w1.size(1) == 32 && b1.numel() == 64 && w2_in.dim() == 2 &&
                  w2_in.size(1) == 64 && b2_in.numel() == w2_in.size(0),
              "nfi: decoder w1 [64,32], b1 [64], w2 [nout,64], b2 [nout] expected");
  const c10::DeviceGuard guard(w1.device());
  Tensor w2 = w2_in.detach(), b2 = b2_in.detach();
  const int64_t rows = w2.size(0);
  if (attention_values < 0) {
    TORCH_CHECK(rows == 11 || rows == 4 || rows == 33,
                "nfi: a decoder output layer of ", rows, " rows is ambiguous: pass attention_values (0 = colour "
                "head [4,64], 1..10 = attention head [N+1,64])");
    attention_values = rows == 4 ? 0 : 10;
  }
  const int32_t nout = rows == 33 ? 33 : 11;
  if (rows != 33) {
    TORCH_CHECK(attention_values <= 10 && rows == (attention_values == 0 ? 4 : attention_values + 1),
                "nfi: decoder output layer of ", rows, " rows does not match attention_values=", attention_values);
    if (rows < 11) {
      const double fill = attention_values == 0 ? 0.0 : -1e30;
      w2 = torch::cat({w2, torch::zeros({11 - rows, w2.size(1)}, w2.options())});
      b2 = torch::cat({b2.reshape({-1}), torch::full({11 - rows}, fill, b2.options())});
    }
  }
  Tensor dec = torch::empty({nfi_decoder_size(nout)}, w1.options());
  const float g1 = scaled ? 1.0f : (float)(1.0 / std::sqrt((double)w1.size(1)));
  const float g2 = scaled ? 1.0f : (float)(1.0 / std::sqrt((double)w2.size(1)));
  Tensor w1c = w1.detach().contiguous(), b1c = b1.detach().contiguous(), w2c = w2.contiguous(), b2c = b2.contiguous();
  check(nfi_decoder_pack_n(w1c.data_ptr<float>(), b1c.data_ptr<float>(), w2c.data_ptr<float>(), b2c.data_ptr<float>(),
                           nout, g1, g2, 1.0f, dec.data_ptr<float>(), stream_of(w1)),
        "nfi_decoder_pack_n");
  return dec;
}

Tensor pack_decoder(const Tensor& w1, const Tensor& b1, const Tensor& w2, const Tensor& b2, int64_t attention_values) {
  return pack_with_gains(w1, b1, w2, b2, false, attention_values);
}

// the attention count of a render / triplane_mlp call: 0 for the colour head, else W2s's logits
int64_t attention_of(const Tensor& W2s, int64_t heads) {
  return (heads & NFI_HEAD_RGB_SIGMOID) ? 0 : W2s.size(0) - 1;
}

// ---- fused render --------------------------------------------------------------------------------
struct RenderCfg {
  int64_t samples, heads, seed;
  bool fine, white, randomize;
  double scene_range, inv_alpha, beta;
};

nfi_render_args render_args(const Tensor& planes_tm, const Tensor& palette, const Tensor& ro, const Tensor& rd,
                            const Tensor& nr, const Tensor& fr, const Tensor& dec, const RenderCfg& c) {
  nfi_render_args a{};
  a.field.planes = planes_tm.data_ptr<float>();
  a.field.sb = planes_tm.stride(0);
  a.field.sq = planes_tm.stride(1);
  a.field.st = planes_tm.stride(3);
  a.field.R = (int32_t)planes_tm.size(2);
  a.field.dec = dec.data_ptr<float>();
  a.field.palette = palette.defined() ? palette.data_ptr<float>() : nullptr;
  a.field.inv_alpha = (float)c.inv_alpha;
  a.field.beta = (float)c.beta;
  a.field.scene_range = (float)c.scene_range;
  a.field.heads = (int32_t)c.heads;
  a.ro = ro.data_ptr<float>();
  a.rd = rd.data_ptr<float>();
  a.near_ = nr.data_ptr<float>();
  a.far_ = fr.data_ptr<float>();
  a.B = (int32_t)planes_tm.size(0);
  a.HW = (int32_t)(ro.size(1) * ro.size(2));
  a.S = (int32_t)c.samples;
  a.fine = c.fine;
  a.white_bg = c.white;
  a.randomize = c.randomize;
  a.W = (int32_t)ro.size(2);
  a.seed = (uint64_t)c.seed;
  a.offset = 0;
  return a;
}

void check_render_inputs(const Tensor& planes_tm, const c10::optional<Tensor>& palette, const Tensor& ro,
                         const Tensor& rd, const Tensor& nr, const Tensor& fr, const Tensor& dec, int64_t heads) {
  for (auto p : {std::make_pair(&planes_tm, "planes_tm"), std::make_pair(&ro, "ro"), std::make_pair(&rd, "rd"),
                 std::make_pair(&nr, "near"), std::make_pair(&fr, "far"), std::make_pair(&dec, "dec")})
    require(*p.first, p.second);
  TORCH_CHECK(planes_tm.dim() == 5 && planes_tm.size(1) == 3 && planes_tm.size(4) == 32 &&
                  planes_tm.size(2) == planes_tm.size(3) && planes_tm.stride(4) == 1 &&
                  planes_tm.stride(2) == planes_tm.size(3) * planes_tm.stride(3),
              "nfi: planes_tm must be texel-major [B,3,R,R,32] with dense rows");
  TORCH_CHECK(ro.dim() == 4 && ro.size(0) == planes_tm.size(0) && ro.size(3) == 3 && ro.is_contiguous() &&
                  rd.is_contiguous() && nr.is_contiguous() && fr.is_contiguous(),
              "nfi: ro, rd [B,H,W,3] and near, far [B,H,W] (contiguous) expected");
  TORCH_CHECK((heads & ~(NFI_HEAD_RGB_SIGMOID | NFI_HEAD_NERF_DENSITY)) == 0,
              "nfi::volume_render: heads 0, NFI_HEAD_RGB_SIGMOID, NFI_HEAD_NERF_DENSITY (the view-direction "
              "closure: nfi.render)");
  TORCH_CHECK((palette && palette->defined()) == !(heads & NFI_HEAD_RGB_SIGMOID),
              "nfi: a palette is required exactly when the colour head is the attention head");
  if (palette && palette->defined()) {
    require(*palette, "palette");
    TORCH_CHECK(palette->sizes() == torch::IntArrayRef({planes_tm.size(0), 10, 3}), "nfi: palette [B,10,3] expected");
  }
}

// volume_render_fwd -> (rgb [B,H,W,3], depth, mask [B,H,W], t, sigma, rgb_s, y, perm, x, tile_counts);
// keep_state false: a forward-only render (the saved-state outputs are empty)
std::vector<Tensor> render_forward_impl(const Tensor& planes_tm, const c10::optional<Tensor>& palette_o, const Tensor& ro,
                                        const Tensor& rd, const Tensor& nr, const Tensor& fr, const Tensor& dec,
                                        int64_t samples, bool fine, bool white, bool randomize, double scene_range,
                                        double inv_alpha, double beta, int64_t heads, int64_t seed,
                                        const c10::optional<Tensor>& u_coarse, const c10::optional<Tensor>& u_fine,
                                        bool keep_state, int64_t offset) {
  check_render_inputs(planes_tm, palette_o, ro, rd, nr, fr, dec, heads);
  const c10::DeviceGuard guard(ro.device());
  const Tensor palette = (palette_o && palette_o->defined()) ? palette_o->contiguous() : Tensor();
  const int64_t B = ro.size(0), H = ro.size(1), W = ro.size(2), n = B * H * W;
  const int64_t N = fine ? 2 * samples : samples;
  for (auto u : {u_coarse, u_fine})
    if (u && u->defined()) {
      require(*u, "u");
      TORCH_CHECK(u->numel() == n * samples && u->is_contiguous(), "nfi: u_coarse / u_fine need B*H*W*S elements");
    }
  auto o = ro.options();
  Tensor rgb = torch::empty({B, H, W, 3}, o), depth = torch::empty({B, H, W}, o), mask = torch::empty({B, H, W}, o);
  Tensor t_s, s_s, c_s, y_s, perm, x_s, tc;
  RenderCfg c{samples, heads, seed, fine, white, randomize, scene_range, inv_alpha, beta};
  nfi_render_args a = render_args(planes_tm, palette, ro, rd, nr, fr, dec, c);
  a.offset = (uint64_t)offset;
  a.u_coarse = fptr(u_coarse);
  a.u_fine = fptr(u_fine);
  a.rgb = rgb.data_ptr<float>();
  a.depth = depth.data_ptr<float>();
  a.mask = mask.data_ptr<float>();
  if (keep_state) {
    t_s = torch::empty({n, N}, o);
    s_s = torch::empty({n, N}, o);
    c_s = torch::empty({n, 3, N}, o);
    y_s = torch::empty({n, 11, N}, o);
    perm = torch::empty({n, N}, o.dtype(torch::kInt16));
    x_s = torch::empty({n * N, 32}, o);
    a.t_saved = t_s.data_ptr<float>();
    a.sigma_saved = s_s.data_ptr<float>();
    a.rgb_saved = c_s.data_ptr<float>();
    a.y_saved = y_s.data_ptr<float>();
    a.perm = perm.data_ptr<int16_t>();
    a.x_saved = x_s.data_ptr<float>();
    const int64_t ntc = nfi_tile_count_size(&a);
    check(ntc < 0 ? -1 : 0, "nfi_tile_count_size");
    tc = torch::empty({ntc}, o.dtype(torch::kInt32));
    a.tile_counts = tc.data_ptr<int32_t>();
  }
  check(nfi_render_forward(&a, stream_of(ro)), "nfi_render_forward");
  auto e = torch::empty({0}, o);
  return {rgb, depth, mask, keep_state ? t_s : e, keep_state ? s_s : e, keep_state ? c_s : e,
          keep_state ? y_s : e, keep_state ? perm : e.to(torch::kInt16), keep_state ? x_s : e,
          keep_state ? tc : e.to(torch::kInt32)};
}

std::vector<Tensor> volume_render_fwd(const Tensor& planes_tm, const c10::optional<Tensor>& palette, const Tensor& ro,
                                      const Tensor& rd, const Tensor& nr, const Tensor& fr, const Tensor& dec,
                                      int64_t samples, bool fine, bool white, bool randomize, double scene_range,
                                      double inv_alpha, double beta, int64_t heads, int64_t seed,
                                      const c10::optional<Tensor>& u_coarse, const c10::optional<Tensor>& u_fine,
                                      bool keep_state) {
  return render_forward_impl(planes_tm, palette, ro, rd, nr, fr, dec, samples, fine, white, randomize, scene_range,
                             inv_alpha, beta, heads, seed, u_coarse, u_fine, keep_state, 0);
}

// volume_render_bwd -> (d_planes (planes_tm's strides), d_palette [B,10,3] or empty, d_ro, d_rd or empty)
std::vector<Tensor> volume_render_bwd(const Tensor& g_rgb_in, const Tensor& g_mask_in, const Tensor& planes_tm,
                                      const c10::optional<Tensor>& palette_o, const Tensor& ro, const Tensor& rd,
                                      const Tensor& nr, const Tensor& fr, const Tensor& dec, int64_t samples, bool fine,
                                      bool white, bool randomize, double scene_range, double inv_alpha, double beta,
                                      int64_t heads, const Tensor& t_s, const Tensor& s_s, const Tensor& c_s,
                                      const Tensor& y_s, const Tensor& perm, const Tensor& x_s, const Tensor& tc,
                                      bool coords) {
  check_render_inputs(planes_tm, palette_o, ro, rd, nr, fr, dec, heads);
  const c10::DeviceGuard guard(ro.device());
  const Tensor palette = (palette_o && palette_o->defined()) ? palette_o->contiguous() : Tensor();
  const int64_t B = ro.size(0), H = ro.size(1), W = ro.size(2), n = B * H * W;
  const int64_t N = fine ? 2 * samples : samples, npl = (N + 63) / 64;
  TORCH_CHECK(t_s.numel() == n * N && x_s.numel() == n * N * 32, "nfi::volume_render_bwd: saved state of another call");
  auto o = ro.options();
  Tensor g_rgb = g_rgb_in.defined() ? g_rgb_in.contiguous() : torch::zeros({n, 3}, o);
  Tensor g_mask = g_mask_in.defined() ? g_mask_in.contiguous() : torch::zeros({n}, o);
  Tensor d_planes = torch::zeros_like(planes_tm);
  TORCH_CHECK(d_planes.strides() == planes_tm.strides(), "nfi: d planes strides differ from the planes view");
  Tensor d_pal_ray = palette.defined() ? torch::empty({n * npl, 30}, o) : Tensor();
  Tensor g_ro = coords ? torch::empty({B, H, W, 3}, o) : Tensor();
  Tensor g_rd = coords ? torch::empty({B, H, W, 3}, o) : Tensor();
  RenderCfg c{samples, heads, 0, fine, white, randomize, scene_range, inv_alpha, beta};
  nfi_render_args a = render_args(planes_tm, palette, ro, rd, nr, fr, dec, c);
  a.t_saved = t_s.data_ptr<float>();
  a.sigma_saved = s_s.data_ptr<float>();
  a.rgb_saved = c_s.data_ptr<float>();
  a.y_saved = y_s.data_ptr<float>();
  a.perm = perm.data_ptr<int16_t>();
  a.x_saved = x_s.data_ptr<float>();
  {
    // torch.use_deterministic_algorithms() (or NFI_DETERMINISTIC) selects the bitwise-reproducible
    // backward: sorted bins, d planes without float atomics (nfi_set_deterministic)
    const char* env = std::getenv("NFI_DETERMINISTIC");
    const bool det = at::globalContext().deterministicAlgorithms() || (env && env[0] && std::strcmp(env, "0") != 0);
    nfi_set_deterministic(det ? 1 : 0);
  }
  const int64_t nbytes = nfi_render_backward_workspace_bytes(&a);
  check(nbytes < 0 ? -1 : 0, "nfi_render_backward_workspace_bytes");
  Tensor ws = torch::empty({nbytes}, o.dtype(torch::kUInt8));
  nfi_render_grad_args g{};
  g.g_rgb = g_rgb.data_ptr<float>();
  g.g_mask = g_mask.data_ptr<float>();
  g.d_planes = d_planes.data_ptr<float>();
  g.d_palette_ray = mptr(d_pal_ray);
  g.g_ro = mptr(g_ro);
  g.g_rd = mptr(g_rd);
  g.tile_counts = tc.numel() ? tc.data_ptr<int32_t>() : nullptr;
  g.workspace = ws.data_ptr<uint8_t>();
  g.workspace_bytes = nbytes;
  void* st = stream_of(ro);
  check(nfi_render_backward(&a, &g, st), "nfi_render_backward");
  Tensor d_pal = torch::empty({0}, o);
  if (palette.defined()) {
    d_pal = torch::empty({B, 30}, o);
    Tensor sws = torch::empty({B * 64 * 30}, o);
    check(nfi_segment_sum(d_pal_ray.data_ptr<float>(), (int32_t)B, (int32_t)(H * W * npl), 30, d_pal.data_ptr<float>(),
                          sws.data_ptr<float>(), st),
          "nfi_segment_sum");
    d_pal = d_pal.view({B, 10, 3});
  }
  auto e = torch::empty({0}, o);
  return {d_planes, d_pal, coords ? g_ro : e, coords ? g_rd : e};
}

struct VolumeRenderFn : public torch::autograd::Function<VolumeRenderFn> {
  static variable_list forward(AutogradContext* ctx, Tensor planes_tm, Tensor palette, Tensor ro, Tensor rd,
                               Tensor nr, Tensor fr, Tensor dec, int64_t samples, bool fine, bool white,
                               bool randomize, double scene_range, double inv_alpha, double beta, int64_t heads,
                               int64_t seed, c10::optional<Tensor> u_coarse, c10::optional<Tensor> u_fine) {
    const bool keep = ctx->needs_input_grad(0) || ctx->needs_input_grad(1) || ctx->needs_input_grad(2) ||
                      ctx->needs_input_grad(3);
    const c10::optional<Tensor> pal = palette.defined() ? c10::optional<Tensor>(palette) : c10::nullopt;
    auto r = volume_render_fwd(planes_tm, pal, ro.contiguous(), rd.contiguous(), nr.contiguous(), fr.contiguous(),
                               dec, samples, fine, white, randomize, scene_range, inv_alpha, beta, heads, seed,
                               u_coarse, u_fine, keep);
    ctx->save_for_backward({planes_tm, palette, ro.contiguous(), rd.contiguous(), nr.contiguous(), fr.contiguous(),
                            dec, r[3], r[4], r[5], r[6], r[7], r[8], r[9]});
    ctx->saved_data["samples"] = samples;
    ctx->saved_data["fine"] = fine;
    ctx->saved_data["white"] = white;
    ctx->saved_data["randomize"] = randomize;
    ctx->saved_data["scene_range"] = scene_range;
    ctx->saved_data["inv_alpha"] = inv_alpha;
    ctx->saved_data["beta"] = beta;
    ctx->saved_data["heads"] = heads;
    ctx->mark_non_differentiable({r[1]});
    return {r[0], r[1], r[2]};
  }

  static variable_list backward(AutogradContext* ctx, variable_list g) {
    auto s = ctx->get_saved_variables();
    auto& d = ctx->saved_data;
    const bool coords = ctx->needs_input_grad(2) || ctx->needs_input_grad(3);
    const c10::optional<Tensor> pal = s[1].defined() ? c10::optional<Tensor>(s[1]) : c10::nullopt;
    const int64_t n = s[2].size(0) * s[2].size(1) * s[2].size(2);
    Tensor g_rgb = g[0].defined() ? g[0].contiguous().view({n, 3}) : Tensor();
    Tensor g_mask = g[2].defined() ? g[2].contiguous().view({n}) : Tensor();
    auto r = volume_render_bwd(g_rgb, g_mask, s[0], pal, s[2], s[3], s[4], s[5], s[6], d["samples"].toInt(),
                               d["fine"].toBool(), d["white"].toBool(), d["randomize"].toBool(),
                               d["scene_range"].toDouble(), d["inv_alpha"].toDouble(), d["beta"].toDouble(),
                               d["heads"].toInt(), s[7], s[8], s[9], s[10], s[11], s[12], s[13], coords);
    variable_list out(18);
    out[0] = r[0];
    out[1] = s[1].defined() ? r[1] : Tensor();
    out[2] = coords ? r[2] : Tensor();
    out[3] = coords ? r[3] : Tensor();
    return out;
  }
};

std::tuple<Tensor, Tensor, Tensor> volume_render(const Tensor& planes_tm, const c10::optional<Tensor>& palette,
                                                 const Tensor& ro, const Tensor& rd, const Tensor& nr, const Tensor& fr,
                                                 const Tensor& dec, int64_t samples, bool fine, bool white,
                                                 bool randomize, double scene_range, double inv_alpha, double beta,
                                                 int64_t heads, int64_t seed, const c10::optional<Tensor>& u_coarse,
                                                 const c10::optional<Tensor>& u_fine) {
  auto r = VolumeRenderFn::apply(planes_tm, palette ? *palette : Tensor(), ro, rd, nr, fr, dec, samples, fine, white,
                                 randomize, scene_range, inv_alpha, beta, heads, seed, u_coarse, u_fine);
  return {r[0], r[1], r[2]};
}

// ---- nerf_utils seams ---------------------------------------------------------------------------
Tensor sample_pdf(const Tensor& bins, const Tensor& weights, int64_t num_samples, bool deterministic,
                  const c10::optional<Tensor>& u, int64_t seed) {
  require(bins, "bins");
  require(weights, "weights");
  const c10::DeviceGuard guard(bins.device());
  TORCH_CHECK(bins.dim() == 2 && weights.dim() == 2 && weights.size(0) == bins.size(0) &&
                  weights.size(1) == bins.size(1) - 1,
              "nfi::sample_pdf: bins [rays, nb] and weights [rays, nb-1] expected");
  const int64_t n = bins.size(0);
  Tensor b = bins.detach().contiguous(), w = weights.detach().contiguous();
  c10::optional<Tensor> uu = u ? c10::optional<Tensor>(u->detach().contiguous()) : c10::nullopt;
  if (uu) TORCH_CHECK(uu->numel() == n * num_samples, "nfi::sample_pdf: u must be [rays, num_samples]");
  Tensor out = torch::empty({n, num_samples}, bins.options());
  check(nfi_sample_pdf(b.data_ptr<float>(), w.data_ptr<float>(), n, (int32_t)bins.size(1), (int32_t)num_samples,
                       deterministic, fptr(uu), (uint64_t)seed, 0, out.data_ptr<float>(), stream_of(bins)),
        "nfi_sample_pdf");
  return out;
}

std::tuple<Tensor, Tensor> compute_near_far_planes(const Tensor& ro, const Tensor& rd, double scene_range) {
  require(ro, "ray_origins");
  require(rd, "ray_directions");
  const c10::DeviceGuard guard(ro.device());
  auto shape = ro.sizes().slice(0, ro.dim() - 1).vec();
  Tensor o = ro.detach().reshape({-1, 3}).contiguous(), d = rd.detach().reshape({-1, 3}).contiguous();
  const int64_t n = o.size(0);
  Tensor nr = torch::empty({n}, ro.options()), fr = torch::empty({n}, ro.options());
  Tensor ws = torch::empty({std::max<int64_t>(1, nfi_near_far_workspace_bytes(n))}, ro.options().dtype(torch::kUInt8));
  check(nfi_near_far(o.data_ptr<float>(), d.data_ptr<float>(), n, (float)scene_range, nr.data_ptr<float>(),
                     fr.data_ptr<float>(), ws.data_ptr<uint8_t>(), stream_of(ro)),
        "nfi_near_far");
  return {nr.view(shape), fr.view(shape)};
}

struct CumprodFn : public torch::autograd::Function<CumprodFn> {
  static Tensor forward(AutogradContext* ctx, Tensor x) {
    require(x, "tensor");
    const c10::DeviceGuard guard(x.device());
    Tensor xc = x.contiguous();
    const int64_t N = xc.size(-1), n = xc.numel() / std::max<int64_t>(N, 1);
    Tensor out = torch::empty_like(xc);
    check(nfi_cumprod_exclusive(xc.data_ptr<float>(), n, (int32_t)N, out.data_ptr<float>(), stream_of(x)),
          "nfi_cumprod_exclusive");
    ctx->save_for_backward({xc});
    return out;
  }
  static variable_list backward(AutogradContext* ctx, variable_list g) {
    Tensor x = ctx->get_saved_variables()[0];
    const int64_t N = x.size(-1), n = x.numel() / N;
    Tensor dx = torch::empty_like(x), gc = g[0].contiguous();
    check(nfi_cumprod_exclusive_backward(x.data_ptr<float>(), gc.data_ptr<float>(), n, (int32_t)N, dx.data_ptr<float>(),
                                         stream_of(x)),
          "nfi_cumprod_exclusive_backward");
    return {dx};
  }
};

Tensor cumprod_exclusive(const Tensor& x) { return CumprodFn::apply(x); }

struct WeightsFn : public torch::autograd::Function<WeightsFn> {
  static Tensor forward(AutogradContext* ctx, Tensor sigma, Tensor rd, Tensor t) {
    require(sigma, "sigma_a");
    require(rd, "ray_directions");
    require(t, "depth_values");
    const c10::DeviceGuard guard(sigma.device());
    Tensor sc = sigma.contiguous(), rc = rd.contiguous(), tcn = t.contiguous();
    const int64_t N = sc.size(-1), n = sc.numel() / N;
    TORCH_CHECK(tcn.sizes() == sc.sizes() && rc.numel() == n * 3 && N <= 1024,
                "nfi::render_volume_density_weights_only: sigma_a [..., N <= 1024], ray_directions [..., 3], "
                "depth_values [..., N] expected");
    Tensor w = torch::empty_like(sc);
    check(nfi_volume_weights_forward(sc.data_ptr<float>(), rc.data_ptr<float>(), tcn.data_ptr<float>(), n, (int32_t)N,
                                     w.data_ptr<float>(), stream_of(sigma)),
          "nfi_volume_weights_forward");
    ctx->save_for_backward({sc, rc, tcn});
    return w;
  }
  static variable_list backward(AutogradContext* ctx, variable_list g) {
    auto s = ctx->get_saved_variables();
    const int64_t N = s[0].size(-1), n = s[0].numel() / N;
    Tensor d_sigma = torch::empty_like(s[0]);
    Tensor d_rd = ctx->needs_input_grad(1) ? torch::empty_like(s[1]) : Tensor();
    Tensor d_t = ctx->needs_input_grad(2) ? torch::empty_like(s[2]) : Tensor();
    Tensor gw = g[0].contiguous();
    check(nfi_volume_weights_backward(s[0].data_ptr<float>(), s[1].data_ptr<float>(), s[2].data_ptr<float>(), n,
                                      (int32_t)N, gw.data_ptr<float>(), d_sigma.data_ptr<float>(), mptr(d_rd),
                                      mptr(d_t), stream_of(s[0])),
          "nfi_volume_weights_backward");
    return {d_sigma, d_rd, d_t};
  }
};

Tensor render_volume_density_weights_only(const Tensor& sigma, const Tensor& ro, const Tensor& rd, const Tensor& t) {
  (void)ro;   // not used by the reference either (nerf_utils.py:166-182)
  return WeightsFn::apply(sigma, rd, t);
}

// ---- SURVEY §8(b) names: the render / per-stage ops on the reference's own layouts -----------------
// planes channel-major [B,3,32,R,R] (generator.py:476-477), the decoder as gain-scaled W1s [64,32], b1,
// W2s [nout,64], b2 (stylegan.py:173-176: W * gain folded on the host).  Each op converts to the
// kernels' layouts (texel-major planes, the packed decoder) on the caller's stream and launches the
// same C-ABI entries volume_render_fwd / _bwd, nfi_composite_*, nfi_sampler_* do.
Tensor to_texel_major(const Tensor& planes) {
  require(planes, "planes");
  TORCH_CHECK(planes.dim() == 5 && planes.size(1) == 3 && planes.size(2) == 32 && planes.size(3) == planes.size(4),
              "nfi: planes [B,3,32,R,R] expected");
  const Tensor p = planes.contiguous();
  const int64_t B = p.size(0), R = p.size(3);
  Tensor tm = torch::empty({B, 3, R, R, 32}, p.options());
  check(nfi_planes_to_texel_major(p.data_ptr<float>(), (int32_t)B, (int32_t)R, tm.data_ptr<float>(), stream_of(p)),
        "nfi_planes_to_texel_major");
  return tm;
}

Tensor to_channel_major(const Tensor& tm) {
  const int64_t B = tm.size(0), R = tm.size(2);
  Tensor p = torch::empty({B, 3, 32, R, R}, tm.options());
  check(nfi_planes_to_channel_major(tm.data_ptr<float>(), (int32_t)B, (int32_t)R, p.data_ptr<float>(), stream_of(tm)),
        "nfi_planes_to_channel_major");
  return p;
}

// render_fwd -> (rgb [B,H,W,3], depth, mask [B,H,W], t_sorted [B,H,W,N], saved_state); N = 2S with fine
// sampling.  saved_state = (planes_tm, dec, t, sigma, rgb_s, y, perm, x, tile_counts): render_bwd's input.
std::tuple<Tensor, Tensor, Tensor, Tensor, std::vector<Tensor>> render_fwd(
    const Tensor& planes, const Tensor& W1s, const Tensor& b1, const Tensor& W2s, const Tensor& b2,
    const c10::optional<Tensor>& palette, double inv_alpha, double beta, const Tensor& ro, const Tensor& rd,
    const Tensor& nr, const Tensor& fr, int64_t S, double scene_range, bool white_bg, bool randomize, int64_t seed,
    int64_t offset, const c10::optional<Tensor>& u_coarse, const c10::optional<Tensor>& u_fine, bool fine,
    int64_t heads) {
  const c10::DeviceGuard guard(planes.device());
  const Tensor tm = to_texel_major(planes);
  const Tensor dec = pack_with_gains(W1s, b1, W2s, b2, true, attention_of(W2s, heads));
  auto r = render_forward_impl(tm, palette, ro.contiguous(), rd.contiguous(), nr.contiguous(), fr.contiguous(), dec, S,
                               fine, white_bg, randomize, scene_range, inv_alpha, beta, heads, seed, u_coarse, u_fine,
                               true, offset);
  const int64_t N = fine ? 2 * S : S;
  Tensor t_sorted = r[3].view({ro.size(0), ro.size(1), ro.size(2), N});
  return {r[0], r[1], r[2], t_sorted, {tm, dec, r[3], r[4], r[5], r[6], r[7], r[8], r[9]}};
}

// render_bwd -> (d_planes [B,3,32,R,R], d_palette [B,10,3] (empty without a palette), d_ro, d_rd [B,H,W,3]
// (empty unless coords))
std::tuple<Tensor, Tensor, Tensor, Tensor> render_bwd(
    const c10::optional<Tensor>& g_rgb, const c10::optional<Tensor>& g_mask, at::TensorList saved,
    const c10::optional<Tensor>& palette, double inv_alpha, double beta, const Tensor& ro, const Tensor& rd,
    const Tensor& nr, const Tensor& fr, int64_t S, double scene_range, bool white_bg, bool randomize, bool fine,
    int64_t heads, bool coords) {
  TORCH_CHECK(saved.size() == 9, "nfi::render_bwd: saved_state is render_fwd's 9-tensor list");
  const c10::DeviceGuard guard(ro.device());
  const int64_t n = ro.size(0) * ro.size(1) * ro.size(2);
  const Tensor gr = (g_rgb && g_rgb->defined()) ? g_rgb->contiguous().view({n, 3}) : Tensor();
  const Tensor gm = (g_mask && g_mask->defined()) ? g_mask->contiguous().view({n}) : Tensor();
  auto r = volume_render_bwd(gr, gm, saved[0], palette, ro.contiguous(), rd.contiguous(), nr.contiguous(),
                             fr.contiguous(), saved[1], S, fine, white_bg, randomize, scene_range, inv_alpha, beta,
                             heads, saved[2], saved[3], saved[4], saved[5], saved[6], saved[7], saved[8], coords);
  return {to_channel_major(r[0]), r[1], r[2], r[3]};
}

// composite_fwd: render_volume_density (nerf_utils.py:125-163) -> (rgb_map [...,3], depth, mask [...],
// weights [...,N]); sigma [...,N], rgb [...,N,3], rd [...,3], t [...,N]
std::tuple<Tensor, Tensor, Tensor, Tensor> composite_fwd(const Tensor& sigma, const Tensor& rgb, const Tensor& rd,
                                                         const Tensor& t, bool white_bg) {
  for (auto p : {std::make_pair(&sigma, "sigma"), std::make_pair(&rgb, "rgb"), std::make_pair(&rd, "rd"),
                 std::make_pair(&t, "t")})
    require(*p.first, p.second);
  const int64_t N = sigma.size(-1), n = sigma.numel() / std::max<int64_t>(N, 1);
  TORCH_CHECK(N >= 1 && N <= 1024 && rgb.numel() == n * N * 3 && rgb.size(-1) == 3 && rd.numel() == n * 3 &&
                  t.sizes() == sigma.sizes(),
              "nfi::composite_fwd: sigma [...,N <= 1024], rgb [...,N,3], rd [...,3], t [...,N] expected");
  const c10::DeviceGuard guard(sigma.device());
  const Tensor sc = sigma.contiguous(), cc = rgb.contiguous(), rc = rd.contiguous(), tc = t.contiguous();
  auto lead = sigma.sizes().slice(0, sigma.dim() - 1).vec();
  auto lead3 = lead;
  lead3.push_back(3);
  auto o = sigma.options();
  Tensor rgb_map = torch::empty(lead3, o), depth = torch::empty(lead, o), mask = torch::empty(lead, o);
  Tensor w = torch::empty_like(sc);
  check(nfi_composite_forward(sc.data_ptr<float>(), cc.data_ptr<float>(), rc.data_ptr<float>(), tc.data_ptr<float>(),
                              n, (int32_t)N, white_bg, rgb_map.data_ptr<float>(), depth.data_ptr<float>(),
                              mask.data_ptr<float>(), w.data_ptr<float>(), stream_of(sigma)),
        "nfi_composite_forward");
  return {rgb_map, depth, mask, w};
}

// composite_bwd -> (d_sigma, d_rgb, d_rd, d_t) in the inputs' shapes; absent gradients count as zero
std::tuple<Tensor, Tensor, Tensor, Tensor> composite_bwd(const Tensor& sigma, const Tensor& rgb, const Tensor& rd,
                                                         const Tensor& t, bool white_bg,
                                                         const c10::optional<Tensor>& g_rgb,
                                                         const c10::optional<Tensor>& g_mask,
                                                         const c10::optional<Tensor>& g_weights) {
  for (auto p : {std::make_pair(&sigma, "sigma"), std::make_pair(&rgb, "rgb"), std::make_pair(&rd, "rd"),
                 std::make_pair(&t, "t")})
    require(*p.first, p.second);
  const int64_t N = sigma.size(-1), n = sigma.numel() / std::max<int64_t>(N, 1);
  TORCH_CHECK(N >= 1 && N <= 1024 && rgb.numel() == n * N * 3 && rd.numel() == n * 3 && t.sizes() == sigma.sizes(),
              "nfi::composite_bwd: sigma [...,N <= 1024], rgb [...,N,3], rd [...,3], t [...,N] expected");
  const c10::DeviceGuard guard(sigma.device());
  const Tensor sc = sigma.contiguous(), cc = rgb.contiguous(), rc = rd.contiguous(), tc = t.contiguous();
  auto o = sigma.options();
  const Tensor gr = (g_rgb && g_rgb->defined()) ? g_rgb->contiguous() : torch::zeros({n, 3}, o);
  const Tensor gm = (g_mask && g_mask->defined()) ? g_mask->contiguous() : torch::zeros({n}, o);
  const Tensor gw = (g_weights && g_weights->defined()) ? g_weights->contiguous() : Tensor();
  TORCH_CHECK(gr.numel() == n * 3 && gm.numel() == n && (!gw.defined() || gw.numel() == n * N),
              "nfi::composite_bwd: gradient shapes differ from the outputs'");
  Tensor d_sigma = torch::empty_like(sc), d_rgb = torch::empty_like(cc), d_rd = torch::empty_like(rc),
         d_t = torch::empty_like(tc);
  check(nfi_composite_backward(sc.data_ptr<float>(), cc.data_ptr<float>(), rc.data_ptr<float>(), tc.data_ptr<float>(),
                               n, (int32_t)N, white_bg, gr.data_ptr<float>(), gm.data_ptr<float>(), mptr(gw),
                               d_sigma.data_ptr<float>(), d_rgb.data_ptr<float>(), d_rd.data_ptr<float>(),
                               d_t.data_ptr<float>(), stream_of(sigma)),
        "nfi_composite_backward");
  return {d_sigma.view(sigma.sizes()), d_rgb.view(rgb.sizes()), d_rd.view(rd.sizes()), d_t.view(t.sizes())};
}

// triplane_mlp: the sampler closure (generator.py:587-681, TriplanarDecoder :301-331) at world points
// x [B,P,3] on planes [B,3,32,R,R]
struct MlpInputs {
  Tensor tm, dec, palette, x;
  nfi_field f;
};

MlpInputs mlp_inputs(const Tensor& planes, const Tensor& W1s, const Tensor& b1, const Tensor& W2s, const Tensor& b2,
                     const c10::optional<Tensor>& palette, const Tensor& x, double inv_alpha, double beta,
                     double scene_range, int64_t heads) {
  require(x, "x");
  TORCH_CHECK(x.dim() == 3 && x.size(0) == planes.size(0) && x.size(2) == 3, "nfi::triplane_mlp: x [B,P,3] expected");
  TORCH_CHECK(heads == 0 || heads == NFI_HEAD_RGB_SIGMOID || heads == NFI_HEAD_NERF_DENSITY ||
                  heads == (NFI_HEAD_RGB_SIGMOID | NFI_HEAD_NERF_DENSITY),
              "nfi::triplane_mlp: heads 0, NFI_HEAD_RGB_SIGMOID, NFI_HEAD_NERF_DENSITY");
  const bool has_pal = palette && palette->defined();
  TORCH_CHECK(has_pal == !(heads & NFI_HEAD_RGB_SIGMOID),
              "nfi: a palette is required exactly when the colour head is the attention head");
  MlpInputs m;
  m.tm = to_texel_major(planes);
  m.dec = pack_with_gains(W1s, b1, W2s, b2, true, attention_of(W2s, heads));
  if (has_pal) {
    require(*palette, "palette");
    TORCH_CHECK(palette->sizes() == torch::IntArrayRef({planes.size(0), 10, 3}), "nfi: palette [B,10,3] expected");
    m.palette = palette->contiguous();
  }
  m.x = x.contiguous();
  m.f = nfi_field{};
  m.f.planes = m.tm.data_ptr<float>();
  m.f.sb = m.tm.stride(0);
  m.f.sq = m.tm.stride(1);
  m.f.st = m.tm.stride(3);
  m.f.R = (int32_t)m.tm.size(2);
  m.f.dec = m.dec.data_ptr<float>();
  m.f.palette = has_pal ? m.palette.data_ptr<float>() : nullptr;
  m.f.inv_alpha = (float)inv_alpha;
  m.f.beta = (float)beta;
  m.f.scene_range = (float)scene_range;
  m.f.heads = (int32_t)heads;
  return m;
}

// triplane_mlp_fwd -> (sigma [B,P], rgb [B,P,3], y [B,P,11] decoder outputs)
std::tuple<Tensor, Tensor, Tensor> triplane_mlp_fwd(const Tensor& planes, const Tensor& W1s, const Tensor& b1,
                                                    const Tensor& W2s, const Tensor& b2,
                                                    const c10::optional<Tensor>& palette, const Tensor& x,
                                                    double inv_alpha, double beta, double scene_range, int64_t heads) {
  const c10::DeviceGuard guard(x.device());
  MlpInputs m = mlp_inputs(planes, W1s, b1, W2s, b2, palette, x, inv_alpha, beta, scene_range, heads);
  const int64_t B = x.size(0), P = x.size(1);
  auto o = x.options();
  Tensor sigma = torch::empty({B, P}, o), rgb = torch::empty({B, P, 3}, o), y = torch::empty({B, P, 11}, o);
  check(nfi_sampler_forward(&m.f, m.x.data_ptr<float>(), (int32_t)B, P, sigma.data_ptr<float>(), rgb.data_ptr<float>(),
                            y.data_ptr<float>(), stream_of(x)),
        "nfi_sampler_forward");
  return {sigma, rgb, y};
}

// triplane_mlp_bwd -> (d_planes [B,3,32,R,R], d_palette [B,10,3] (empty without a palette), d_x [B,P,3])
std::tuple<Tensor, Tensor, Tensor> triplane_mlp_bwd(const Tensor& planes, const Tensor& W1s, const Tensor& b1,
                                                    const Tensor& W2s, const Tensor& b2,
                                                    const c10::optional<Tensor>& palette, const Tensor& x,
                                                    double inv_alpha, double beta, double scene_range, int64_t heads,
                                                    const c10::optional<Tensor>& g_sigma,
                                                    const c10::optional<Tensor>& g_rgb,
                                                    const c10::optional<Tensor>& g_y) {
  const c10::DeviceGuard guard(x.device());
  MlpInputs m = mlp_inputs(planes, W1s, b1, W2s, b2, palette, x, inv_alpha, beta, scene_range, heads);
  const int64_t B = x.size(0), P = x.size(1);
  auto o = x.options();
  auto grad = [&](const c10::optional<Tensor>& g, int64_t k, const char* name) {
    if (!g || !g->defined()) return Tensor();
    require(*g, name);
    TORCH_CHECK(g->numel() == B * P * k, "nfi::triplane_mlp_bwd: ", name, " has the wrong size");
    return g->contiguous();
  };
  const Tensor gs = grad(g_sigma, 1, "g_sigma"), gr = grad(g_rgb, 3, "g_rgb"), gy = grad(g_y, 11, "g_y");
  Tensor d_tm = torch::zeros_like(m.tm), d_x = torch::empty({B, P, 3}, o);
  const int64_t chunks = nfi_sampler_chunks((int32_t)B, P);
  Tensor d_part = m.palette.defined() ? torch::empty({chunks, 30}, o) : Tensor();
  void* st = stream_of(x);
  check(nfi_sampler_backward(&m.f, m.x.data_ptr<float>(), (int32_t)B, P, gs.defined() ? gs.data_ptr<float>() : nullptr,
                             gr.defined() ? gr.data_ptr<float>() : nullptr, gy.defined() ? gy.data_ptr<float>() : nullptr,
                             d_tm.data_ptr<float>(), mptr(d_part), d_x.data_ptr<float>(), st),
        "nfi_sampler_backward");
  Tensor d_pal = torch::empty({0}, o);
  if (m.palette.defined()) {
    d_pal = torch::empty({B, 30}, o);
    Tensor ws = torch::empty({B * 64 * 30}, o);
    check(nfi_segment_sum(d_part.data_ptr<float>(), (int32_t)B, (int32_t)(chunks / B), 30, d_pal.data_ptr<float>(),
                          ws.data_ptr<float>(), st),
          "nfi_segment_sum");
    d_pal = d_pal.view({B, 10, 3});
  }
  return {to_channel_major(d_tm), d_pal, d_x};
}

// ---- Meta kernels (shape propagation for the tracing front ends; no computation) ------------------
std::vector<Tensor> volume_render_fwd_meta(const Tensor& planes_tm, const c10::optional<Tensor>&, const Tensor& ro,
                                           const Tensor&, const Tensor&, const Tensor&, const Tensor&, int64_t samples,
                                           bool fine, bool, bool, double, double, double, int64_t, int64_t,
                                           const c10::optional<Tensor>&, const c10::optional<Tensor>&,
                                           bool keep_state) {
  const int64_t B = ro.size(0), H = ro.size(1), W = ro.size(2), n = B * H * W;
  const int64_t N = fine ? 2 * samples : samples;
  auto o = ro.options();
  auto e = [&](std::vector<int64_t> s, c10::ScalarType t = torch::kFloat) {
    return torch::empty(keep_state ? s : std::vector<int64_t>{0}, o.dtype(t));
  };
  return {torch::empty({B, H, W, 3}, o), torch::empty({B, H, W}, o), torch::empty({B, H, W}, o), e({n, N}),
          e({n, N}), e({n, 3, N}), e({n, 11, N}), e({n, N}, torch::kInt16), e({n * N, 32}),
          // the library's own rule (beams included when it was built with NFI_BEAM_SAMPLES)
          e({nfi_tile_count_size_shape((int32_t)B, (int32_t)planes_tm.size(2), (int32_t)H, (int32_t)W, (int32_t)N)},
            torch::kInt32)};
}

std::vector<Tensor> volume_render_bwd_meta(const Tensor&, const Tensor&, const Tensor& planes_tm,
                                           const c10::optional<Tensor>& palette, const Tensor& ro, const Tensor&,
                                           const Tensor&, const Tensor&, const Tensor&, int64_t, bool, bool, bool,
                                           double, double, double, int64_t, const Tensor&, const Tensor&,
                                           const Tensor&, const Tensor&, const Tensor&, const Tensor&, const Tensor&,
                                           bool coords) {
  auto o = ro.options();
  const int64_t B = ro.size(0), H = ro.size(1), W = ro.size(2);
  return {torch::empty_like(planes_tm),
          (palette && palette->defined()) ? torch::empty({B, 10, 3}, o) : torch::empty({0}, o),
          coords ? torch::empty({B, H, W, 3}, o) : torch::empty({0}, o),
          coords ? torch::empty({B, H, W, 3}, o) : torch::empty({0}, o)};
}

}  // namespace

TORCH_LIBRARY(nfi, m) {
  m.def("rays(Tensor cam, Tensor? focal, Tensor? center, Tensor? bbox, int H, int W, float scene_range) "
        "-> (Tensor, Tensor, Tensor, Tensor)");
  m.def("pack_decoder(Tensor w1, Tensor b1, Tensor w2, Tensor b2, int attention_values=-1) -> Tensor");
  m.def("volume_render(Tensor planes_tm, Tensor? palette, Tensor ro, Tensor rd, Tensor near, Tensor far, "
        "Tensor dec, int samples, bool fine, bool white_background, bool randomize, float scene_range, "
        "float inv_alpha, float beta, int heads, int seed, Tensor? u_coarse=None, Tensor? u_fine=None) "
        "-> (Tensor, Tensor, Tensor)");
  m.def("volume_render_fwd(Tensor planes_tm, Tensor? palette, Tensor ro, Tensor rd, Tensor near, Tensor far, "
        "Tensor dec, int samples, bool fine, bool white_background, bool randomize, float scene_range, "
        "float inv_alpha, float beta, int heads, int seed, Tensor? u_coarse, Tensor? u_fine, bool keep_state) "
        "-> Tensor[]");
  m.def("volume_render_bwd(Tensor g_rgb, Tensor g_mask, Tensor planes_tm, Tensor? palette, Tensor ro, Tensor rd, "
        "Tensor near, Tensor far, Tensor dec, int samples, bool fine, bool white_background, bool randomize, "
        "float scene_range, float inv_alpha, float beta, int heads, Tensor t_saved, Tensor sigma_saved, "
        "Tensor rgb_saved, Tensor y_saved, Tensor perm, Tensor x_saved, Tensor tile_counts, bool coords) "
        "-> Tensor[]");
  m.def("sample_pdf(Tensor bins, Tensor weights, int num_samples, bool deterministic=False, Tensor? u=None, "
        "int seed=0) -> Tensor");
  m.def("compute_near_far_planes(Tensor ray_origins, Tensor ray_directions, float scene_range) -> (Tensor, Tensor)");
  m.def("cumprod_exclusive(Tensor tensor) -> Tensor");
  m.def("render_volume_density_weights_only(Tensor sigma_a, Tensor ray_origins, Tensor ray_directions, "
        "Tensor depth_values) -> Tensor");
  m.def("render_fwd(Tensor planes, Tensor W1s, Tensor b1, Tensor W2s, Tensor b2, Tensor? palette, float inv_alpha, "
        "float beta, Tensor ro, Tensor rd, Tensor near, Tensor far, int S, float scene_range, bool white_bg, "
        "bool randomize, int seed, int offset, Tensor? u_coarse=None, Tensor? u_fine=None, bool fine=True, "
        "int heads=0) -> (Tensor, Tensor, Tensor, Tensor, Tensor[])");
  m.def("render_bwd(Tensor? grad_rgb, Tensor? grad_mask, Tensor[] saved_state, Tensor? palette, float inv_alpha, "
        "float beta, Tensor ro, Tensor rd, Tensor near, Tensor far, int S, float scene_range, bool white_bg, "
        "bool randomize, bool fine=True, int heads=0, bool coords=True) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("composite_fwd(Tensor sigma, Tensor rgb, Tensor rd, Tensor t, bool white_bg) "
        "-> (Tensor, Tensor, Tensor, Tensor)");
  m.def("composite_bwd(Tensor sigma, Tensor rgb, Tensor rd, Tensor t, bool white_bg, Tensor? g_rgb, Tensor? g_mask, "
        "Tensor? g_weights=None) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("triplane_mlp_fwd(Tensor planes, Tensor W1s, Tensor b1, Tensor W2s, Tensor b2, Tensor? palette, Tensor x, "
        "float inv_alpha, float beta, float scene_range, int heads=0) -> (Tensor, Tensor, Tensor)");
  m.def("triplane_mlp_bwd(Tensor planes, Tensor W1s, Tensor b1, Tensor W2s, Tensor b2, Tensor? palette, Tensor x, "
        "float inv_alpha, float beta, float scene_range, int heads, Tensor? g_sigma, Tensor? g_rgb, "
        "Tensor? g_y=None) -> (Tensor, Tensor, Tensor)");
}

// the autograd-carrying ops decompose into their torch::autograd::Function (which records the graph)
TORCH_LIBRARY_IMPL(nfi, CompositeImplicitAutograd, m) {
  m.impl("rays", &rays);
  m.impl("volume_render", &volume_render);
  m.impl("cumprod_exclusive", &cumprod_exclusive);
  m.impl("render_volume_density_weights_only", &render_volume_density_weights_only);
}

// HIP devices are the CUDA dispatch key in PyTorch-ROCm
TORCH_LIBRARY_IMPL(nfi, CUDA, m) {
  m.impl("pack_decoder", &pack_decoder);
  m.impl("volume_render_fwd", &volume_render_fwd);
  m.impl("volume_render_bwd", &volume_render_bwd);
  m.impl("sample_pdf", &sample_pdf);
  m.impl("compute_near_far_planes", &compute_near_far_planes);
  m.impl("render_fwd", &render_fwd);
  m.impl("render_bwd", &render_bwd);
  m.impl("composite_fwd", &composite_fwd);
  m.impl("composite_bwd", &composite_bwd);
  m.impl("triplane_mlp_fwd", &triplane_mlp_fwd);
  m.impl("triplane_mlp_bwd", &triplane_mlp_bwd);
}

TORCH_LIBRARY_IMPL(nfi, Meta, m) {
  m.impl("volume_render_fwd", &volume_render_fwd_meta);
  m.impl("volume_render_bwd", &volume_render_bwd_meta);
}
