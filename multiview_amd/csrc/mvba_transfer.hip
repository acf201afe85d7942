// mvba_transfer.hip — host hand-over of an evaluation (the ceres::CostFunction
// surface, include/mvba/ceres_surface.h; Problem::Evaluate's Jacobian layout).
//
// K1 leaves residuals and Jacobian entries in column planes in device order
// (one plane per Jacobian row). Ceres wants, per residual block
// in AddResidualBlock order (rig_calibrator.cc:1695-1699), the row-major
// 2 x size_b Jacobian of every non-NULL block (Ceres 1.14 CostFunction::Evaluate
// [ext]), with the loss corrector applied. k_rows turns the planes into those
// rows on the device so the host receives ONE contiguous DMA:
//   * a wave stages T slots x (2 + jac_rows) values in LDS (plane reads: 64
//     consecutive doubles per instruction);
//   * then writes each slot's row contiguously at its offset (64 lanes = 512
//     consecutive bytes per store), Cauchy corrector sqrt(rho') applied
//     (Ceres' Corrector for rho'' < 0 [ext]); the loss itself is computed one
//     slot per lane.
// Two row layouts:
//   full   : jac_rows doubles per residual in AddResidualBlock order
//            (MVBA_JAC_BASE_* positions), blocks that are constant for the
//            residual zero-filled (mvba_evaluate);
//   packed : per slot, only the blocks in its transfer mask, in block-position
//            order, rows in device (frame) order so a wave's rows are one
//            contiguous range of whole lines (mvba_evaluate_packed; skips the
//            columns nobody asked for; offsets locate each residual's row).
// The same kernel serves BracketedDepthError blocks (3 residuals, 7 blocks,
// depth_to_image 7 or 12 wide; rig_calibrator.cc:522-609): a RowsLayout says
// how many residual rows, where each block's plane rows start and how wide the
// blocks are (one block per family has a per-slot width: distortion K /
// depth_to_image n).
// HBM traffic is 2x the row bytes (read planes, write rows): small next to the
// PCIe copy that follows (DESIGN.md §5 "Host transfer").
#include "mvba_internal.h"

namespace mvba {

struct RowsArgs {
  const double* res;          // [nres][ld]
  const double* J;            // [jac_rows][ld] or null (residuals only)
  int64_t ld, slot0, nslots;  // slots [slot0, nslots)
  int32_t jac_rows;
  int32_t nres;               // residual rows per block (2 or 3)
  int32_t nblocks;            // parameter blocks per residual block (8 or 7)
  int32_t var_block;          // the block whose width is per slot
  int32_t base[8];            // first plane row of block b
  int32_t size[8];            // width of block b (var_block: per slot)
  int32_t tile;               // slots per wave (power of two <= 64)
  int32_t log2_tile;
  int32_t pitch;              // LDS doubles per staged slot (odd)
  double cauchy_c;            // 0: no loss
  const int64_t* order;       // slot -> insertion index (-1 padding)
  const uint8_t* written;     // slot -> blocks the evaluation kernel wrote
  const int16_t* varsize;     // slot -> width of var_block
  const uint8_t* xmask;       // packed: slot -> transferred blocks; null = full layout
  const int64_t* xoff;        // packed: slot -> row offset (doubles)
  double* out_res;            // [nres N] insertion order, corrected
  double* out_cost;           // [N] insertion order (0.5 rho or 0.5 |r|^2), nullable
  double* out_rows;           // rows, nullable
};

__global__ void __launch_bounds__(64) k_rows(RowsArgs a) {
  // Ceres computes the loss and corrector on the CPU without fused multiply-adds;
  // keep every product and sum separately rounded so the rows match bit for bit.
#pragma clang fp contract(off)
  extern __shared__ double tile[];
  const int lane = threadIdx.x;
  const int T = a.tile, P = a.pitch, R = a.nres, NB = a.nblocks, LT = a.log2_tile;
  const int64_t p0 = a.slot0 + (int64_t)blockIdx.x * T;
  const int nrows = a.J ? R + a.jac_rows : R;
  // stage: T slots x nrows values; consecutive lanes read consecutive slots of a
  // plane. Eight loads are issued before their LDS stores (a plain loop waits
  // for each load before the next, the store being in between).
  const int total = T * nrows;
  for (int base = lane; base < total; base += 8 * 64) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int idx = base + 64 * u;
      const int row = idx >> LT, sl = idx & (T - 1);
      const int64_t p = p0 + sl;
      v[u] = 0.0;
      if (idx < total && p < a.nslots) v[u] = row < R ? a.res[row * a.ld + p] : a.J[(int64_t)(row - R) * a.ld + p];
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int idx = base + 64 * u;
      if (idx < total) tile[(idx & (T - 1)) * P + (idx >> LT)] = v[u];
    }
  }
  // per-slot records, one slot per lane, loaded once for the whole tile (the
  // slot loop below reads them with lane broadcasts)
  int64_t my_i = -1, my_off = 0;
  int my_w = 0, my_vs = 0, my_xm = 0;
  if (lane < T && p0 + lane < a.nslots) {
    const int64_t p = p0 + lane;
    my_i = a.order[p];
    my_w = a.written[p];
    my_vs = a.varsize[p];
    if (a.xmask) {
      my_xm = a.xmask[p];
      my_off = a.xoff[p];
    }
  }
  __syncthreads();
  // loss, corrected residuals and cost: one slot per lane
  double my_sr = 1.0;
  if (my_i >= 0) {
    const double* t = tile + lane * P;
    double s2 = 0.0;
    for (int q = 0; q < R; q++) s2 += t[q] * t[q];
    double ci = 0.5 * s2;
    if (a.cauchy_c > 0.0) {
      // Ceres 1.14 CauchyLoss + Corrector [ext] (b = 1/c)
      const double b = 1.0 / a.cauchy_c;
      const double sum = 1.0 + s2 * a.cauchy_c;
      ci = 0.5 * (b * log(sum));
      my_sr = sqrt(fmax(2.2250738585072014e-308, 1.0 / sum));
    }
    for (int q = 0; q < R; q++) a.out_res[R * my_i + q] = t[q] * my_sr;
    if (a.out_cost) a.out_cost[my_i] = ci;
  }
  if (!a.out_rows || !a.J) return;
  // Row table: output entry k of a slot's row comes from plane row rowtab[k]
  // (-1: a constant block, zero). It depends only on (written blocks, variable
  // width, transfer mask), which a frame's slots share, so it is rebuilt only
  // when that key changes (about once per wave), not per slot and entry.
  short* rowtab = reinterpret_cast<short*>(tile + (size_t)T * P);
  int key_prev = -1, len = 0;
  for (int s = 0; s < T; s++) {
    const int64_t i = __shfl(my_i, s, 64);
    if (i < 0) continue;  // padding slot or past the last slot (wave-uniform)
    const int wmask = __shfl(my_w, s, 64);
    const int vs = __shfl(my_vs, s, 64);
    const int xm = a.xmask ? __shfl(my_xm, s, 64) : 0xFF;
    const int key = wmask | (xm << 8) | (vs << 16);
    if (key != key_prev) {
      __syncthreads();  // (one wave per block) the previous table's reads are done
      if (!a.xmask) {
        len = a.jac_rows;
        for (int k = lane; k < len; k += 64) {
          int b = 0;  // the block owning plane row k: the last one starting at or before k
#pragma unroll
          for (int q = 1; q < 8; q++)
            if (q < NB && k >= a.base[q]) b = q;
          const int w = (b == a.var_block) ? vs : a.size[b];
          rowtab[k] = (short)((((wmask >> b) & 1) && k < a.base[b] + R * w) ? k : -1);
        }
      } else {
        len = 0;
#pragma unroll
        for (int b = 0; b < 8; b++)
          if (b < NB && ((xm >> b) & 1)) len += R * (b == a.var_block ? vs : a.size[b]);
        for (int k = lane; k < len; k += 64) {
          // walk the transferred blocks to the one holding packed entry k
          int start = 0, row = 0, b_of = 0;
          bool found = false;
#pragma unroll
          for (int b = 0; b < 8; b++) {
            if (b >= NB || !((xm >> b) & 1)) continue;
            const int n = R * (b == a.var_block ? vs : a.size[b]);
            if (!found && k < start + n) {
              row = a.base[b] + (k - start);
              b_of = b;
              found = true;
            }
            start += n;
          }
          rowtab[k] = (short)(((wmask >> b_of) & 1) ? row : -1);
        }
      }
      __syncthreads();
      key_prev = key;
    }
    const double* t = tile + s * P + R;
    const double sr = __shfl(my_sr, s, 64);
    double* dst = a.xmask ? a.out_rows + __shfl(my_off, s, 64) : a.out_rows + i * (int64_t)a.jac_rows;
    for (int k = lane; k < len; k += 64) {
      const int r = rowtab[k];
      dst[k] = r >= 0 ? t[r] * sr : 0.0;
    }
  }
}

}  // namespace mvba

extern "C" hipError_t mvba_launch_rows(const double* res, const double* J, int64_t ld, int64_t slot0, int64_t nslots,
                                       const mvba_rows_layout* L, double cauchy_c, const int64_t* order,
                                       const uint8_t* written, const int16_t* varsize, const uint8_t* xmask,
                                       const int64_t* xoff, double* out_res, double* out_cost, double* out_rows,
                                       hipStream_t s) {
  if (nslots <= slot0) return hipSuccess;
  mvba::RowsArgs a;
  a.res = res;
  a.J = J;
  a.ld = ld;
  a.slot0 = slot0;
  a.nslots = nslots;
  a.jac_rows = L->jac_rows;
  a.nres = L->nres;
  a.nblocks = L->nblocks;
  a.var_block = L->var_block;
  for (int b = 0; b < 8; b++) {
    a.base[b] = L->base[b];
    a.size[b] = L->size[b];
  }
  const int nrows = J ? L->nres + L->jac_rows : L->nres;
  // tile: slots per wave (power of two, <= 64) within 20 KB of LDS, so several
  // waves share a CU and hide each other's plane reads
  int T = 64;
  while (T > 1 && (size_t)T * (size_t)(nrows | 1) * sizeof(double) > 20480) T /= 2;
  a.tile = T;
  a.log2_tile = 0;
  while ((1 << a.log2_tile) < T) a.log2_tile++;
  a.pitch = nrows | 1;
  a.cauchy_c = cauchy_c;
  a.order = order;
  a.written = written;
  a.varsize = varsize;
  a.xmask = xmask;
  a.xoff = xoff;
  a.out_res = out_res;
  a.out_cost = out_cost;
  a.out_rows = out_rows;
  // staged tile + the row table (short per Jacobian row)
  const size_t lds = (size_t)T * (size_t)a.pitch * sizeof(double) + sizeof(short) * (size_t)(L->jac_rows + 8);
  const int64_t nblk = (nslots - slot0 + T - 1) / T;
  hipLaunchKernelGGL(mvba::k_rows, dim3((unsigned)nblk), dim3(64), lds, s, a);
  return hipGetLastError();
}
