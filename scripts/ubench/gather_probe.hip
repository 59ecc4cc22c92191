// Probe (not product code): the forward's tap gather alone, over the forward's own merged sample
// depths, at the forward's occupancy — the time the tap stream needs with nothing else in the
// kernel (no decoder, no scans, no saved state).  Compiled with the render source included, so it
// runs exactly the product's gather_features (quad layout, load records, buffer loads):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics \
//         -I nerf-from-image_amd/csrc scripts/ubench/gather_probe.hip nerf-from-image_amd/csrc/nfi_rays.hip \
//         -o scripts/ubench/libgather_probe.so
// Driven by scripts/gather_probe.py (bench inputs, HIP-event timing).
#include "nfi_render.hip"

namespace nfi {

// one wave per ray (ray_of_block order, as render_fwd_kernel), its merged samples in chunks of 64
// (a.t_saved [rays][N]); each sample's 32 gathered features are summed into out[r*N + i]
__global__ void __launch_bounds__(256, NFI_FWD_OCC) gather_probe_kernel(nfi_render_args a, float* out) {
  __shared__ __attribute__((aligned(16))) float lds[4 * XTILE];
  const int wv = threadIdx.x >> 6, l = lane_id();
  const long long nrays = (long long)a.B * a.HW;
  const long long r = ray_of_block(blockIdx.x, 4, a) + wv;
  if (r >= nrays) return;
  const int N = a.fine ? 2 * a.S : a.S;
  float* X = lds + wv * XTILE;
  RayCtx R;
  load_ray(a, r, R);
  const PlaneView pv{a.field.planes + (long long)R.b * a.field.sb, (int)a.field.sq, (int)a.field.st,
                     a.field.R};
  for (int e = 0; e * 64 < N; ++e) {
    const int npts = min(64, N - e * 64);
    const float t = a.t_saved[r * N + e * 64 + min(l, npts - 1)];
    PointP P;
    point_params(R.o, R.d, t, a.field.scene_range, pv.R, P);
    gather_features(pv, P, npts, X);
    wave_lds_sync();
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NC / 4; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(X + l * XS + 4 * k);
      s += (v.x + v.y) + (v.z + v.w);
    }
    if (l < npts) out[r * N + e * 64 + l] = s;
    wave_lds_sync();
  }
}

}  // namespace nfi

extern "C" int32_t nfi_gather_probe(const nfi_render_args* a, float* out, hipStream_t s) {
  const long long nrays = (long long)a->B * a->HW;
  nfi::gather_probe_kernel<<<(unsigned)((nrays + 3) / 4), 256, 0, s>>>(*a, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
