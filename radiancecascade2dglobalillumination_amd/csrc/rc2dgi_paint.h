// rc2dgi_paint.h -- on-device scene producer: raylib 5.5 rectangles and circles
// rasterized into colorRT / emissiveRT the way RenderScene / RedrawSceneToRTs paint them
// (RC2DGI.cs:224-264, 528-545).  See rc2dgi_paint.hip.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/rc2dgi.h"
#include "rc2dgi_kernels.h"

namespace rc2dgi {

// device copies of the primitive setup, grown on demand (owned by the context)
struct PaintBuffers {
  void *prims = nullptr;  // PaintPrim[]
  void *edges = nullptr;  // PaintTri[]
  size_t prim_cap = 0, tri_cap = 0;
  void release();
  ~PaintBuffers() { release(); }
};

// BeginTextureMode(dst); [ClearBackground(clear)]; draw prims[0..n); EndTextureMode.
// dst: W x H float4 render texture (pitch in texels), GL row order; u8: an RGBA8 texture (values
// k * (1/255), 8-bit blends).  Synchronous w.r.t. the host arrays (they are copied before
// returning); the raster runs on `st`.
hipError_t paint_prims(float4 *dst, int W, int H, int pitch, bool u8, const unsigned char *clear,
                       const rc2dgi_prim *prims, int n, PaintBuffers &buf, hipStream_t st);

}  // namespace rc2dgi
