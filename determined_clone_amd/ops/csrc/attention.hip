// Flash attention (forward + backward) on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), bf16 in/out,
// fp32 softmax statistics, causal or full, head dim 64 / 128.
//
// Replaces the fused softmax/attention CUDA kernels the reference's GPT-NeoX DeepSpeedTrial gets
// from DeepSpeed/apex (examples/deepspeed/gpt_neox). Inputs are strided [B, S, H, D] or
// [B, H, S, D] views (last dim contiguous), so the model can pass slices of its fused QKV
// projection without copies.
//
// Forward, one workgroup = 4 wave64 = 64 query rows of one (batch, head):
//   Q fragments live in VGPRs for the whole kernel; per 64-key tile K is staged row-major and V
//   transposed into LDS (padded rows, 16-B ds_read_b128 fragment reads), S = Q K^T (16x16x32
//   MFMA), online softmax in the exp2 domain with 16-lane shuffle row reductions, P goes through a
//   per-wave LDS tile to become the A operand of O += P V. Writes O and the row log-sum-exp.
// Backward (FlashAttention-2 ordering), one workgroup = 64 keys; dK/dV accumulate in VGPRs while
//   the workgroup sweeps the query tiles; recomputed P^T = exp2(S^T - LSE), dP^T = V dO^T,
//   dS^T = P^T (dP^T - rowsum(dO*O)); dQ partials are added into an fp32 buffer with float atomics.
#include <cstdlib>
#include <string>
#include <type_traits>

#include "common.h"

namespace dca {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 64;   // query rows per forward block / keys per backward block
constexpr int kPad = 8;     // LDS row padding (elements) to break power-of-two bank strides
// Row padding of tiles that are only read transposed (ds_read_b64_tr_b16: per 32-lane group, 4 rows
// x 64 B): rows D + 32 elements apart sit 16 banks apart mod 64, so the 4 rows never share a bank
// (with kPad two of them do: 2-way conflicts). Tiles read row-wise by ds_read_b128 keep kPad (its
// lane groups span rows 0-3, 12-15, 20-27, conflict-free at a 144-B stride but not at this one).
constexpr int kTrPad = 32;
constexpr float kRescaleLog2 = 8.f;  // forward: deferred-max threshold (log2 units)

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 load8(const uint16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

__device__ __forceinline__ bf16x8 zero8() {
  uint4 z = make_uint4(0, 0, 0, 0);
  return __builtin_bit_cast(bf16x8, z);
}

__device__ __forceinline__ uint16_t to_bf16(float f) { return static_cast<uint16_t>(f2bf_bits(f)); }
__device__ __forceinline__ float from_bf16(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q / columns 4p..4p+3 of a 4x16
// block; lane i receives column i (4 rows) -- a transposed fragment read straight from a row-major
// LDS tile. Needs all 64 lanes active.
__device__ __forceinline__ s16x4 tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(p));
}

__device__ __forceinline__ bf16x8 cat8(s16x4 a, s16x4 b) {
  const s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// 8 consecutive accumulator registers [base, base+8) -> bf16 MFMA fragment.
__device__ __forceinline__ bf16x8 pack8(const f32x16& x, int base) {
  uint4 u;
  u.x = pack_bf16x2(x[base + 0], x[base + 1]);
  u.y = pack_bf16x2(x[base + 2], x[base + 3]);
  u.z = pack_bf16x2(x[base + 4], x[base + 5]);
  u.w = pack_bf16x2(x[base + 6], x[base + 7]);
  return __builtin_bit_cast(bf16x8, u);
}

// O *= alpha for the deferred-max rescale, one v_mul_f32 per register. Written as plain f32x16
// arithmetic the compiler emits 8 v_pk_mul_f32 per accumulator (packed f32 VALU costs ~22-26
// extra cycles each beside MFMAs on gfx950 -- an anti-lever) AND if-converts the wave-uniform
// `if (__any(upd))` around it, so every sub-tile paid 16 packed multiplies (ISA census of this
// file, round 4). volatile asm keeps the multiplies single-issue and inside the branch.
__device__ __forceinline__ void rescale16(f32x16& a, float s) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float t = a[i];
    asm volatile("v_mul_f32 %0, %1, %2" : "=v"(t) : "v"(t), "v"(s));
    a[i] = t;
  }
}

// v_exp_f32 directly (inputs are finite or -inf; no denormal range fix-up needed)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// max / sum of a value with the same value in lane i^32 (the other half-wave): one
// v_permlane32_swap (a VALU lane exchange) instead of a ds_bpermute round trip through the LDS
// unit and its lgkmcnt wait (guide T12). The swap leaves lanes 0-31 with (own, partner) and lanes
// 32-63 with (partner, own): either order gives the same max / sum. fmax via asm: fmaxf would add
// two canonicalising v_max on the swap results.
__device__ __forceinline__ float half_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  float o;
  asm("v_max_f32 %0, %1, %2" : "=v"(o) : "v"(__uint_as_float(r[0])), "v"(__uint_as_float(r[1])));
  return o;
}
__device__ __forceinline__ float half_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Epilogue store of one row-per-lane-pair accumulator set (T21): lane r holds columns 8k..8k+3 and
// lane r+32 columns 8k+4..8k+7 of group k. One v_permlane32_swap per dword of the group pair
// (k, k+1) leaves the lower lane with all of group k and the upper lane with all of group k+1, so
// each lane writes 16 contiguous bytes: half the store instructions of the 8-byte form. Every lane
// must execute the swaps (all 64 active); `ok` guards only the stores (same for both lanes of a row).
template <int D>
__device__ __forceinline__ void store_rows(uint16_t* row, const f32x16 (&acc)[D / 32], float mul,
                                           int hf, bool ok) {
#pragma unroll
  for (int n = 0; n < D / 32; ++n)
#pragma unroll
    for (int g = 0; g < 4; g += 2) {
      uint32_t ax = pack_bf16x2(acc[n][4 * g] * mul, acc[n][4 * g + 1] * mul);
      uint32_t ay = pack_bf16x2(acc[n][4 * g + 2] * mul, acc[n][4 * g + 3] * mul);
      uint32_t bx = pack_bf16x2(acc[n][4 * g + 4] * mul, acc[n][4 * g + 5] * mul);
      uint32_t by = pack_bf16x2(acc[n][4 * g + 6] * mul, acc[n][4 * g + 7] * mul);
      const auto rx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
      const auto ry = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
      if (ok) *reinterpret_cast<uint4*>(row + 32 * n + 8 * g + 8 * hf) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
    }
}

struct Strides {
  int64_t b, h, s;  // element strides; d stride is 1
};

// XCD-aware workgroup order (guide T1). Consecutive workgroup ids are dealt round-robin to the 8
// XCDs, each with its own L2, so the query (or key) blocks of one (batch, head) -- which all stream
// the same K/V (or Q/dO) tiles -- would be spread over 8 L2s and every tile fetched 8 times from
// HBM / MALL. With remap, each XCD gets a contiguous range of grid positions (the bijective form,
// valid for any grid size): the blocks of a (batch, head) share one L2.
//
// order 2 (heaviest first, causal): additionally, each XCD walks its (batch, head) pairs
// x-slowest -- every pair's x = 0 block (the largest causal extent: the last query block of the
// forward / dQ pass, the first key block of the dK/dV pass) before any pair's x = 1 -- so the
// light blocks fill the tail of the launch instead of heavy ones (longest-processing-time-first).
// A pair's blocks then no longer run together; the K/V (Q/dO) re-reads come from the Infinity
// Cache. Needs (batch * heads) % 8 == 0, else order 1.
struct Blk {
  int x, y, z;
};
__device__ __forceinline__ Blk xcd_block(int order) {
  if (order == 0) return {static_cast<int>(blockIdx.x), static_cast<int>(blockIdx.y), static_cast<int>(blockIdx.z)};
  const int nx = gridDim.x, ny = gridDim.y;
  const int n = nx * ny * gridDim.z;
  const int l = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  const int nbh = ny * static_cast<int>(gridDim.z);
  if (order == 2 && nbh % 8 == 0) {
    const int per = nbh / 8;          // (batch, head) pairs per XCD
    const int p = l / 8;              // dispatch position within this XCD's stream
    const int bh = (l % 8) * per + p % per;
    return {p / per, bh % ny, bh / ny};
  }
  const int xcd = l % 8, q = n / 8, r = n % 8;
  const int v = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + l / 8;
  return {v % nx, (v / nx) % ny, v / (nx * ny)};
}

// Register double buffer for a pair of [ROWS][D] tiles (K and V): fetch() issues the HBM loads of
// the NEXT tile before the current tile's MFMAs, store() writes them to LDS after the barrier.
// Loads go through buffer descriptors whose range ends after row n_rows - 1: rows past it (the
// tail tile, padded keys) come back as zeros from the hardware range check -- no per-chunk
// branches, and 32-bit lane offsets computed once instead of 64-bit addresses per tile (the
// host checks that (Sk + ROWS) * row stride stays below 2^31 bytes).
template <int D, int ROWS = 64, int VPAD = kPad, int NT = 256>
struct KVPrefetch {
  static constexpr int CPR = D / 8;
  static constexpr int PER = ROWS * CPR / NT;  // 16-B chunks per thread per tensor
  static constexpr int N = 2 * PER;
  uint4 reg[N];
  uint32_t voff[N];  // byte offset of this lane's chunk j in a tile starting at row 0
  __amdgpu_buffer_rsrc_t kr, vr;
  uint32_t kstep, vstep;  // bytes per row
  __device__ __forceinline__ void init(const uint16_t* __restrict__ kb, Strides ks,
                                       const uint16_t* __restrict__ vb, Strides vs, int n_rows) {
    kstep = static_cast<uint32_t>(ks.s) * 2u;
    vstep = static_cast<uint32_t>(vs.s) * 2u;
    kr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(kb), 0,
                                           static_cast<int>((n_rows - 1) * kstep + 2u * D), 0x00020000);
    vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(vb), 0,
                                           static_cast<int>((n_rows - 1) * vstep + 2u * D), 0x00020000);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int cc = threadIdx.x + NT * (j % PER);
      const int rr = cc / CPR, d0 = (cc % CPR) * 8;
      voff[j] = static_cast<uint32_t>(rr) * (j < PER ? kstep : vstep) + 2u * d0;
    }
  }
  __device__ __forceinline__ void fetch(int r0) {
    const uint32_t ko = static_cast<uint32_t>(r0) * kstep, vo = static_cast<uint32_t>(r0) * vstep;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const auto t = __builtin_amdgcn_raw_buffer_load_b128(j < PER ? kr : vr,
                                                           voff[j] + (j < PER ? ko : vo), 0, 0);
      reg[j] = __builtin_bit_cast(uint4, t);
    }
  }
  __device__ __forceinline__ void store(uint16_t* Ks, uint16_t* Vs) const {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int cc = threadIdx.x + NT * (j % PER);
      const int rr = cc / CPR, d0 = (cc % CPR) * 8;
      *reinterpret_cast<uint4*>(j >= PER ? Vs + rr * (D + VPAD) + d0 : Ks + rr * (D + kPad) + d0) = reg[j];
    }
  }
};

// Direct-to-LDS staging of the K / V (Q / dO) tiles (buffer_load_dwordx4 ... lds, guide §5
// "glds"): no VGPR round trip, no ds_write, and a 2-stage LDS ring so the next tile streams in
// during the current tile's MFMAs with ONE barrier per tile. A wave instruction writes 1 KB of LDS
// (lane l at +16 l), so rows are unpadded and conflict-free reads come from an XOR swizzle of the
// 16-B chunks instead: the chunk stored at (row, p) is source chunk p ^ f(row), and readers address
// chunk c of a row at c ^ f(row). One f serves both read patterns of a tile:
//  * ds_read_b128 row reads (16 lanes = 16 consecutive rows at one chunk) need 16 distinct bank
//    positions: f(row) must be a permutation over 16 rows (per row parity on 128-B rows);
//  * ds_read_b64_tr_b16 (32 lanes = 4 consecutive rows x a 4-chunk quad) need the 4 rows' quads
//    apart: f's bit 2 (D 64: rows 0/2 and 1/3 share a bank line) or bits 2-3 (D 128) must differ.
// D 64 (128-B rows): f = 4 ((row >> 1) & 1) + ((row >> 2) & 3); D 128 (256-B rows):
// f = 4 (row & 3) + ((row >> 2) & 3).
// Issued as inline asm: with the builtin, hipcc treats every later ds_read_b64_tr_b16 as possibly
// reading the in-flight DMA bytes and puts an s_waitcnt vmcnt(0) in front of the V reads, which
// serialises the next tile's loads with this tile's MFMAs. hipcc does not count these loads: the
// loop waits for them itself (vmcnt(0) + barrier). M0 is saved and restored inside the statement.
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t rsrc, uint32_t voff, void* lds_dst) {
  const uint32_t la = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) void*)(lds_dst)));
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(la), "s"(rsrc)
      : "memory");
}
template <int D>
__device__ __forceinline__ int swz(int row) {
  return D == 128 ? 4 * (row & 3) + ((row >> 2) & 3) : 4 * ((row >> 1) & 1) + ((row >> 2) & 3);
}
// element offset of 16-B chunk c of `row` in a swizzled tile row
template <int D>
__device__ __forceinline__ int swz_off(int row, int c) { return 8 * (c ^ swz<D>(row)); }
// this lane's ds_read_b64_tr_b16 element offset in column block n of a transposed fragment read
// whose rows start at a multiple of 16 (the lane reads row 4 hf + tr_row, +8 for the second half)
template <int D>
__device__ __forceinline__ int tr_off(int lane, int n, bool plus8) {
  const int r = lane & 31, hf = lane >> 5, tr_row = (r & 15) >> 2;
  return swz_off<D>(4 * hf + tr_row + (plus8 ? 8 : 0), 4 * n + 2 * (r >> 4) + ((r & 3) >> 1)) + 4 * (r & 1);
}

template <int D, int ROWS, int NW = 4>
struct KVDma {
  static constexpr int CPR = D / 8;           // 16-B chunks per row
  static constexpr int RPI = 64 / CPR;        // rows per wave instruction (1 KB)
  static constexpr int IPW = ROWS / RPI / NW; // instructions per wave per tensor per tile
  __amdgpu_buffer_rsrc_t kr, vr;
  uint32_t kstep, vstep;
  uint32_t ko[IPW], vo[IPW];
  __device__ __forceinline__ void init(const uint16_t* __restrict__ kb, Strides ks,
                                       const uint16_t* __restrict__ vb, Strides vs, int n_rows,
                                       int w, int lane) {
    kstep = static_cast<uint32_t>(ks.s) * 2u;
    vstep = static_cast<uint32_t>(vs.s) * 2u;
    // rows past n_rows read as zeros (buffer range check)
    kr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(kb), 0,
                                           static_cast<int>((n_rows - 1) * kstep + 2u * D), 0x00020000);
    vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(vb), 0,
                                           static_cast<int>((n_rows - 1) * vstep + 2u * D), 0x00020000);
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int row = (w * IPW + i) * RPI + lane / CPR, pc = lane % CPR;
      ko[i] = static_cast<uint32_t>(row) * kstep + 16u * static_cast<uint32_t>(pc ^ swz<D>(row));
      vo[i] = static_cast<uint32_t>(row) * vstep + 16u * static_cast<uint32_t>(pc ^ swz<D>(row));
    }
  }
  // new tensor bases (same strides): the dK/dV kernel moves on to the next query head
  __device__ __forceinline__ void set_base(const uint16_t* __restrict__ kb, const uint16_t* __restrict__ vb,
                                           int n_rows) {
    kr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(kb), 0,
                                           static_cast<int>((n_rows - 1) * kstep + 2u * D), 0x00020000);
    vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(vb), 0,
                                           static_cast<int>((n_rows - 1) * vstep + 2u * D), 0x00020000);
  }
  __device__ __forceinline__ void issue(uint16_t* Kst, uint16_t* Vst, int r0, int w) const {
    const uint32_t kb0 = static_cast<uint32_t>(r0) * kstep, vb0 = static_cast<uint32_t>(r0) * vstep;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      blds16(kr, ko[i] + kb0, Kst + (w * IPW + i) * 512);
      blds16(vr, vo[i] + vb0, Vst + (w * IPW + i) * 512);
    }
  }
};

// ------------------------------------------------------------------------------------ forward
// One workgroup = 4 waves x 32 queries = 128 query rows of one (batch, head). Per 64-key LDS tile,
// each wave computes S^T = K Q^T as 32x32 tiles with v_mfma_f32_32x32x16_bf16 so that the KEY is in
// the registers and the QUERY on the lane: the softmax row statistics are lane-local (16 registers
// + one exchange with lane^32), and P^T -- still in registers -- is directly the B operand of
// O^T += V^T P^T (no LDS round trip for P). V^T fragments come from the row-major V tile through
// ds_read_b64_tr_b16 (hardware transpose), so K and V are staged exactly as they arrive from HBM.
//
// (Measured and removed: row sums on the matrix core, -2..+1 %; 64 query rows per wave, -10..-24 %;
// the timing-only ablations that chose the DMA ring -- profiles/round5_attention_dma_ring_ab.txt,
// round4_attention_msum_ab.txt.)
template <int D, bool CAUSAL, int KT, bool PIPE, bool DMA = false>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
    uint16_t* __restrict__ o, float* __restrict__ lse, int Sq, int Sk, int H, Strides qs,
    Strides ks, Strides vs, Strides os, float scale_log2, int order, const int* __restrict__ kvlen, int G) {
  // KT = keys per LDS tile (one barrier pair per tile), consumed in 32-key MFMA sub-tiles
  constexpr int QB = 128;      // queries per workgroup
  constexpr int RS = D + kPad; // LDS row stride (elements)
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Ks = smem;           // [KT][RS]
  // V tile: read only transposed -- the conflict-free kTrPad stride for D = 128 (+5-14%); D = 64
  // measured 1-3% slower with it at S 1024-2048 (profiles/round3_attention_vtile_pad_ab.txt)
  constexpr int VPAD = D == 128 ? kTrPad : kPad;
  constexpr int RSV = D + VPAD;
  uint16_t* Vs = Ks + KT * RS;   // [KT][RSV]
  const int lane = threadIdx.x & 63;
  // wave index in an SGPR: the causal extent checks below are uniform branches
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const Blk blk = xcd_block(order);
  const int b = blk.z, h = blk.y;
  // key padding: keys at or past kvlen[b] are masked like keys past Sk (>= 1 key kept)
  if (kvlen) Sk = min(Sk, max(kvlen[b], 1));
  // heaviest (largest causal extent) query blocks first
  const int q_blk = (CAUSAL ? (gridDim.x - 1 - blk.x) : blk.x) * QB;
  const int q0 = q_blk + w * 32;
  const int my_q = q0 + r;
  const uint16_t* qb = q + b * qs.b + h * qs.h;
  // grouped-query attention: G consecutive query heads share K/V head h / G
  const uint16_t* kb = k + b * ks.b + (h / G) * ks.h;
  const uint16_t* vb = v + b * vs.b + (h / G) * vs.h;

  bf16x8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s)
    qf[s] = my_q < Sq ? load8(qb + static_cast<int64_t>(my_q) * qs.s + 16 * s + 8 * hf) : zero8();
  f32x16 oacc[D / 32];
#pragma unroll
  for (int n = 0; n < D / 32; ++n) oacc[n] = zero16();
  float m = -INFINITY, l = 0.f;
  const int k_end = CAUSAL ? min(Sk, q_blk + QB) : Sk;
  // tr-read lane address pieces (see T10: lane 4q+p of a 16-lane group -> row q, cols 4p..4p+3)
  const int tr_row = (r & 15) >> 2;
  const int tr_col = 16 * (r >> 4) + 4 * (r & 3);
  // LDS fragment addresses: padded rows (register-staged tiles) or the swizzled unpadded rows of
  // the DMA ring (KVDma); kx / vx: this lane's element offsets inside a row
  constexpr int KRS = DMA ? D : RS, VRS = DMA ? D : RSV;
  int kx[D / 16], vx[D / 32], vx8[D / 32];
#pragma unroll
  for (int s2 = 0; s2 < D / 16; ++s2) kx[s2] = DMA ? swz_off<D>(r, 2 * s2 + hf) : 16 * s2 + 8 * hf;
#pragma unroll
  for (int n = 0; n < D / 32; ++n) {
    vx[n] = DMA ? tr_off<D>(lane, n, false) : 32 * n + tr_col;
    vx8[n] = DMA ? tr_off<D>(lane, n, true) : 32 * n + tr_col;
  }
  KVPrefetch<D, KT, VPAD> pf;
  KVDma<D, KT> dma;
  if constexpr (DMA) {
    dma.init(kb, ks, vb, vs, Sk, w, lane);
    dma.issue(smem, smem + KT * D, 0, w);
  } else {
    pf.init(kb, ks, vb, vs, Sk);
    pf.fetch(0);
  }
  int stage = 0;
  for (int kt = 0; kt < k_end; kt += KT) {
    if constexpr (DMA) {
      // this tile's loads (issued one tile ago) landed for this wave; the barrier publishes every
      // wave's part and retires the previous tile's reads of the other stage
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      Ks = smem + stage * 2 * KT * D;
      Vs = Ks + KT * D;
      if (kt + KT < k_end) dma.issue(smem + (stage ^ 1) * 2 * KT * D, smem + (stage ^ 1) * 2 * KT * D + KT * D, kt + KT, w);
      stage ^= 1;
    } else {
      __syncthreads();
      pf.store(Ks, Vs);
      __syncthreads();
      if (kt + KT < k_end) pf.fetch(kt + KT);
    }
    if constexpr (PIPE) {
      // online softmax of one sub-tile's scores and O^T += V^T P^T
      auto softmax_pv = [&](f32x16 sc, const int sub, const int kb0, const bool need_mask) {
        // sc[i]: key = kb0 + (i&3) + 8(i>>2) + 4hf, query = my_q
        // row max on the RAW scores (scale > 0 commutes with max); the scale is folded into the
        // exponent's FMA below -- one VALU op per score instead of a multiply and a subtract
        if (need_mask) {
  #pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = kb0 + (i & 3) + 8 * (i >> 2) + 4 * hf;
            sc[i] = (key >= Sk || (CAUSAL && key > my_q)) ? -INFINITY : sc[i];
          }
        }
        float mx = -INFINITY;
  #pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, sc[i]);
        mx = half_max(mx);
        // deferred max (T13): the running max m moves only when a score exceeds it by more than
        // kRescaleLog2 (p <= 2^kRescaleLog2 meanwhile: exact in the fp32 accumulators, 8 bits of
        // headroom in the bf16 P), so the D/2-multiply rescale of O and l runs on a few sub-tiles
        // per row instead of on every max increase. Per lane (= query row): the factor that scales
        // this lane's l is the one that scales its O accumulators.
        const float mcand = mx * scale_log2;
        const bool upd = mcand > m + kRescaleLog2;
        const float mnew = upd ? mcand : m;
        const float mref = mnew == -INFINITY ? 0.f : mnew;
        const float alpha = upd ? fast_exp2(m - mref) : 1.f;
        float rs = 0.f;
  #pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = fast_exp2(fmaf(sc[i], scale_log2, -mref));
          sc[i] = p;
          rs += p;
        }
        rs = half_sum(rs);
        l = l * alpha + rs;
        m = mnew;
        if (__any(upd)) {
  #pragma unroll
          for (int n = 0; n < D / 32; ++n) rescale16(oacc[n], alpha);
        }
        const bf16x8 p0 = pack8(sc, 0), p1 = pack8(sc, 8);
  #pragma unroll
        for (int n = 0; n < D / 32; ++n) {
  #pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const uint16_t* base = Vs + (32 * sub + 16 * s2 + 4 * hf + tr_row) * VRS;
            oacc[n] = mfma32(cat8(tr_read(base + vx[n]), tr_read(base + 8 * VRS + vx8[n])), s2 ? p1 : p0, oacc[n]);
          }
        }
      };
      // wave-uniform: every key of the tile exists and precedes every query of this wave
      if (kt + KT <= Sk && (!CAUSAL || kt + KT - 1 <= q0)) {
        // pairs of sub-tiles: both score products are issued before the first softmax, so the
        // second one's MFMAs run in the matrix pipe under the first softmax's VALU work
#pragma unroll
        for (int sub = 0; sub < KT / 32; sub += 2) {
          // both sub-tiles' K fragments read up front, their two independent MFMA chains
          // interleaved (back-to-back MFMAs without waiting on each other's results)
          bf16x8 ka[D / 16], kb2[D / 16];
  #pragma unroll
          for (int s = 0; s < D / 16; ++s) {
            ka[s] = load8(Ks + (32 * sub + r) * KRS + kx[s]);
            kb2[s] = load8(Ks + (32 * sub + 32 + r) * KRS + kx[s]);
          }
          f32x16 sa = zero16(), sb = zero16();
  #pragma unroll
          for (int s = 0; s < D / 16; ++s) {
            sa = mfma32(ka[s], qf[s], sa);
            sb = mfma32(kb2[s], qf[s], sb);
          }
          // schedule: every fragment read issued before the first MFMA (one LDS wait)
          __builtin_amdgcn_sched_group_barrier(0x100, D / 8, 0);
          __builtin_amdgcn_sched_group_barrier(0x8, D / 8, 0);
          softmax_pv(sa, sub, kt + 32 * sub, false);
          softmax_pv(sb, sub + 1, kt + 32 * sub + 32, false);
        }
        continue;
      }
    }
#pragma unroll
    for (int sub = 0; sub < KT / 32; ++sub) {
      const int kb0 = kt + 32 * sub;
      if (kb0 >= k_end) break;
      if (CAUSAL && kb0 > q0 + 31) break;  // wave-uniform: the rest of this tile is masked
      // every K fragment read issued before the first MFMA: one LDS wait instead of one per MFMA
      bf16x8 kf[D / 16];
#pragma unroll
      for (int s = 0; s < D / 16; ++s) kf[s] = load8(Ks + (32 * sub + r) * KRS + kx[s]);
      f32x16 sc = zero16();
#pragma unroll
      for (int s = 0; s < D / 16; ++s) sc = mfma32(kf[s], qf[s], sc);
      __builtin_amdgcn_sched_group_barrier(0x100, D / 16, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, D / 16, 0);
      // sc[i]: key = kb0 + (i&3) + 8(i>>2) + 4hf, query = my_q
      const bool need_mask = (kb0 + 32 > Sk) || (CAUSAL && kb0 + 31 > q0);
      // one wave-uniform branch around the whole mask (selects, no per-score branches: written
      // inside the max loop, the compiler emitted a scalar test + branch per score on every tile)
      if (need_mask) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kb0 + (i & 3) + 8 * (i >> 2) + 4 * hf;
          sc[i] = (key >= Sk || (CAUSAL && key > my_q)) ? -INFINITY : sc[i];
        }
      }
      // row max on the RAW scores (scale > 0 commutes with max); the scale is folded into the
      // exponent's FMA below -- one VALU op per score instead of a multiply and a subtract
      float mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) mx = fmaxf(mx, sc[i]);
      mx = half_max(mx);
      // deferred max (T13): the running max m moves only when a score exceeds it by more than
      // kRescaleLog2 (p <= 2^kRescaleLog2 meanwhile: exact in the fp32 accumulators, 8 bits of
      // headroom in the bf16 P), so the D/2-multiply rescale of O and l runs on a few sub-tiles
      // per row instead of on every max increase. Per lane (= query row): the factor that scales
      // this lane's l is the one that scales its O accumulators.
      const float mcand = mx * scale_log2;
      const bool upd = mcand > m + kRescaleLog2;
      const float mnew = upd ? mcand : m;
      const float mref = mnew == -INFINITY ? 0.f : mnew;
      const float alpha = upd ? fast_exp2(m - mref) : 1.f;
      float rs = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = fast_exp2(fmaf(sc[i], scale_log2, -mref));
        sc[i] = p;
        rs += p;
      }
      rs = half_sum(rs);
      l = l * alpha + rs;
      m = mnew;
      if (__any(upd)) {
#pragma unroll
        for (int n = 0; n < D / 32; ++n) rescale16(oacc[n], alpha);
      }
      const bf16x8 p0 = pack8(sc, 0), p1 = pack8(sc, 8);
#pragma unroll
      for (int n = 0; n < D / 32; ++n) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const uint16_t* base = Vs + (32 * sub + 16 * s2 + 4 * hf + tr_row) * VRS;
          oacc[n] = mfma32(cat8(tr_read(base + vx[n]), tr_read(base + 8 * VRS + vx8[n])), s2 ? p1 : p0, oacc[n]);
        }
      }
    }
  }
  // 8-byte stores here: the widened form (store_rows) measured -2..-3% on this kernel at S >= 2048
  // (+1.5% at S 1024), +2.5-4% on the backward kernels (profiles/round3_attention_epilogue_ab.txt)
  if (my_q < Sq) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    uint16_t* orow = o + b * os.b + h * os.h + static_cast<int64_t>(my_q) * os.s;
#pragma unroll
    for (int n = 0; n < D / 32; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 pk;
        pk.x = pack_bf16x2(oacc[n][4 * g] * inv, oacc[n][4 * g + 1] * inv);
        pk.y = pack_bf16x2(oacc[n][4 * g + 2] * inv, oacc[n][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + 32 * n + 8 * g + 4 * hf) = pk;
      }
    if (hf == 0)
      lse[(static_cast<int64_t>(b) * H + h) * Sq + my_q] = l > 0.f ? m + log2f(l) : INFINITY;
  }
}

// ------------------------------------------------------------------------------------ backward
// Two kernels, no atomics (FlashAttention-2 style split, MI355X layouts):
//  * attn_bwd_dq_kernel: one workgroup = 128 queries (4 waves x 32). Computes delta = rowsum(dO*O)
//    in its prologue (written for the dK/dV kernel), then sweeps key tiles like the forward:
//    S^T = K Q^T and dP^T = V dO^T with the key in registers / query on the lane, dS^T lane-local,
//    dQ^T += K^T dS^T with K^T fragments from ds_read_b64_tr_b16 -> dQ written once, in bf16.
//  * attn_bwd_dkdv_kernel: one workgroup = 128 keys (4 waves x 32); dK^T / dV^T accumulate in
//    registers while the workgroup sweeps 32-query tiles (double-buffered through registers so the
//    next tile's HBM loads overlap the current tile's MFMAs). S and dP have the key on the lane, so
//    P and dS are directly the B operands of dV^T += dO^T P and dK^T += Q^T dS (A operands by
//    transposed LDS reads of the row-major Q / dO tiles).
template <int D, bool CAUSAL, int KT, bool PIPE, bool DMA = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
    const uint16_t* __restrict__ o, const uint16_t* __restrict__ dO, const float* __restrict__ lse,
    float* __restrict__ delta, uint16_t* __restrict__ dq, int Sq, int Sk, int H, Strides qs,
    Strides ks, Strides vs, Strides os, Strides dos, Strides dqs, float scale_log2, float scale,
    int order, const int* __restrict__ kvlen, int G) {
  // KT = keys per LDS tile (one barrier pair per tile), consumed in 32-key MFMA sub-tiles
  constexpr int QB = 128;
  constexpr int RS = D + kPad;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Ks = smem;
  uint16_t* Vs = Ks + KT * RS;
  const int lane = threadIdx.x & 63;
  // wave index in an SGPR: every per-wave condition below (causal extents, masking) is a
  // uniform branch instead of per-lane exec masking
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const Blk blk = xcd_block(order);
  const int b = blk.z, h = blk.y;
  // key padding: keys at or past kvlen[b] are masked like keys past Sk (>= 1 key kept)
  if (kvlen) Sk = min(Sk, max(kvlen[b], 1));
  const int q_blk = (CAUSAL ? (gridDim.x - 1 - blk.x) : blk.x) * QB;
  const int q0 = q_blk + w * 32;
  const int my_q = q0 + r;
  const bool q_ok = my_q < Sq;
  const uint16_t* kb = k + b * ks.b + (h / G) * ks.h;  // grouped-query: K/V head h / G
  const uint16_t* vb = v + b * vs.b + (h / G) * vs.h;
  const int64_t bh = static_cast<int64_t>(b) * H + h;

  bf16x8 qf[D / 16], dof[D / 16];
  float dsum = 0.f;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const int d0 = 16 * s + 8 * hf;
    qf[s] = q_ok ? load8(q + b * qs.b + h * qs.h + static_cast<int64_t>(my_q) * qs.s + d0) : zero8();
    dof[s] = q_ok ? load8(dO + b * dos.b + h * dos.h + static_cast<int64_t>(my_q) * dos.s + d0) : zero8();
    if (q_ok) {
      const bf16x8 of = load8(o + b * os.b + h * os.h + static_cast<int64_t>(my_q) * os.s + d0);
#pragma unroll
      for (int j = 0; j < 8; ++j) dsum += static_cast<float>(of[j]) * static_cast<float>(dof[s][j]);
    }
  }
  dsum = half_sum(dsum);
  if (q_ok && hf == 0) delta[bh * Sq + my_q] = dsum;
  const float lq = q_ok ? lse[bh * Sq + my_q] : INFINITY;
  f32x16 dqacc[D / 32];
#pragma unroll
  for (int n = 0; n < D / 32; ++n) dqacc[n] = zero16();
  const int tr_row = (r & 15) >> 2;
  const int tr_col = 16 * (r >> 4) + 4 * (r & 3);
  const int k_end = CAUSAL ? min(Sk, q_blk + QB) : Sk;
  // LDS fragment addresses (see attn_fwd_kernel): padded rows or the swizzled DMA ring
  constexpr int KRS = DMA ? D : RS;
  int kx[D / 16], tx[D / 32], tx8[D / 32];
#pragma unroll
  for (int s2 = 0; s2 < D / 16; ++s2) kx[s2] = DMA ? swz_off<D>(r, 2 * s2 + hf) : 16 * s2 + 8 * hf;
#pragma unroll
  for (int n = 0; n < D / 32; ++n) {
    tx[n] = DMA ? tr_off<D>(lane, n, false) : 32 * n + tr_col;
    tx8[n] = DMA ? tr_off<D>(lane, n, true) : 32 * n + tr_col;
  }
  KVPrefetch<D, KT> pf;
  KVDma<D, KT> dma;
  if constexpr (DMA) {
    dma.init(kb, ks, vb, vs, Sk, w, lane);
    dma.issue(smem, smem + KT * D, 0, w);
  } else {
    pf.init(kb, ks, vb, vs, Sk);
    pf.fetch(0);
  }
  int stage = 0;
  for (int kt = 0; kt < k_end; kt += KT) {
    if constexpr (DMA) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of tile kt landed
      __builtin_amdgcn_s_barrier();                       // everyone's; the other stage is free
      asm volatile("" ::: "memory");
      Ks = smem + stage * 2 * KT * D;
      Vs = Ks + KT * D;
      if (kt + KT < k_end)
        dma.issue(smem + (stage ^ 1) * 2 * KT * D, smem + (stage ^ 1) * 2 * KT * D + KT * D, kt + KT, w);
      stage ^= 1;
    } else {
      __syncthreads();
      pf.store(Ks, Vs);
      __syncthreads();
      if (kt + KT < k_end) pf.fetch(kt + KT);
    }
    // S^T = K Q^T and dP^T = V dO^T for the 32-key sub-tile `sub` of the staged tile
    auto sdp = [&](const int sub, f32x16& sc, f32x16& dp) {
      sc = zero16();
      dp = zero16();
      if constexpr (D == 64) {  // fragments preloaded (see the forward)
        bf16x8 kfr[D / 16], vfr[D / 16];
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          kfr[s] = load8(Ks + (32 * sub + r) * KRS + kx[s]);
          vfr[s] = load8(Vs + (32 * sub + r) * KRS + kx[s]);
        }
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          sc = mfma32(kfr[s], qf[s], sc);
          dp = mfma32(vfr[s], dof[s], dp);
        }
      } else {
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          sc = mfma32(load8(Ks + (32 * sub + r) * KRS + kx[s]), qf[s], sc);
          dp = mfma32(load8(Vs + (32 * sub + r) * KRS + kx[s]), dof[s], dp);
        }
      }
    };
    // dS^T = P^T (dP^T - delta) and dQ^T += K^T dS^T
    auto finish = [&](auto masked, f32x16 sc, f32x16 dp, const int sub, const int kb0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = fast_exp2(fmaf(sc[i], scale_log2, -lq));
        if constexpr (decltype(masked)::value) {
          const int key = kb0 + (i & 3) + 8 * (i >> 2) + 4 * hf;
          p = (key >= Sk || (CAUSAL && key > my_q)) ? 0.f : p;
        }
        dp[i] = p * (dp[i] - dsum);  // the softmax scale is applied once to dQ at the end
      }
      const bf16x8 s0 = pack8(dp, 0), s1 = pack8(dp, 8);
#pragma unroll
      for (int n = 0; n < D / 32; ++n)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const uint16_t* base = Ks + (32 * sub + 16 * s2 + 4 * hf + tr_row) * KRS;
          dqacc[n] = mfma32(cat8(tr_read(base + tx[n]), tr_read(base + 8 * KRS + tx8[n])), s2 ? s1 : s0, dqacc[n]);
        }
    };
    auto sub_tile = [&](auto masked, const int sub, const int kb0) {
      f32x16 sc, dp;
      sdp(sub, sc, dp);
      finish(masked, sc, dp, sub, kb0);
    };
    if constexpr (PIPE) {
      // wave-uniform: every key of the tile exists and precedes every query of this wave. Both
      // sub-tiles' score / dP products are issued before the first softmax gradient, so the
      // second pair's MFMAs run in the matrix pipe under the first one's VALU work.
      if (kt + KT <= Sk && (!CAUSAL || kt + KT - 1 <= q0)) {
#pragma unroll
        for (int sub = 0; sub < KT / 32; sub += 2) {
          f32x16 sa, da, sb, db;
          sdp(sub, sa, da);
          sdp(sub + 1, sb, db);
          finish(std::false_type{}, sa, da, sub, kt + 32 * sub);
          finish(std::false_type{}, sb, db, sub + 1, kt + 32 * sub + 32);
        }
        continue;
      }
    }
#pragma unroll
    for (int sub = 0; sub < KT / 32; ++sub) {
      const int kb0 = kt + 32 * sub;
      if (kb0 >= k_end) break;
      if (CAUSAL && kb0 > q0 + 31) break;
      // wave-uniform; D = 128 keeps one (masked) copy: two copies exceed the VGPR budget
      if (D == 128 || (kb0 + 32 > Sk) || (CAUSAL && kb0 + 31 > q0))
        sub_tile(std::true_type{}, sub, kb0);
      else
        sub_tile(std::false_type{}, sub, kb0);
    }
  }
  store_rows<D>(dq + b * dqs.b + h * dqs.h + static_cast<int64_t>(my_q) * dqs.s, dqacc, scale, hf, q_ok);
}

// QT = queries staged per LDS tile (one barrier pair per tile); each wave consumes it in 32-query
// MFMA sub-tiles, so QT = 64 halves the barriers and staging passes per MFMA of QT = 32.
template <int D, bool CAUSAL, int QT>
__global__ __launch_bounds__(256, D == 64 ? 2 : 1) void attn_bwd_dkdv_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
    const uint16_t* __restrict__ dO, const float* __restrict__ lse, const float* __restrict__ delta,
    uint16_t* __restrict__ dk, uint16_t* __restrict__ dv, int Sq, int Sk, int H, Strides qs,
    Strides ks, Strides vs, Strides dos, Strides dks, Strides dvs, float scale_log2, float scale,
    int order, const int* __restrict__ kvlen, int G) {
  constexpr int KB = 128;
  static_assert(QT == 32 || QT == 64, "query tile");
  // padded rows (the XOR-swizzled unpadded layout of KVDma removed the 0.92 bank-conflict cycles per
  // LDS instruction but measured neutral: profiles/round5_attention_dma_ring_ab.txt)
  constexpr int RS = D + kPad;
  constexpr int CPR = D / 8;                 // 16-byte chunks per row
  constexpr int NPF = 2 * QT * CPR / 256;    // prefetched chunks per thread (Q and dO tiles)
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Qs = smem;            // [QT][RS]
  uint16_t* dOs = Qs + QT * RS;   // [QT][RS]
  float* lse_s = reinterpret_cast<float*>(dOs + QT * RS);
  float* del_s = lse_s + QT;
  const int lane = threadIdx.x & 63;
  // wave index in an SGPR: every per-wave condition below (causal extents, masking) is a
  // uniform branch instead of per-lane exec masking
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const Blk blk = xcd_block(order);
  const int b = blk.z, h = blk.y;
  const int SkT = Sk;  // rows of dK/dV to write (padded keys get zeros)
  // key padding: keys at or past kvlen[b] are masked like keys past Sk (>= 1 key kept)
  if (kvlen) Sk = min(Sk, max(kvlen[b], 1));
  const int k_blk = blk.x * KB;
  const int kw0 = k_blk + 32 * w;
  const int my_key = kw0 + r;
  // h is the K/V head (grid y runs over H / G of them); its G query heads h*G .. h*G+G-1 are swept
  // one after another below, dK / dV summing over all of them in the same registers
  const uint16_t* qb = q;
  const uint16_t* dob = dO;
  int64_t bh = 0;

  bf16x8 kf[D / 16], vf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const bool ok = my_key < Sk;
    kf[s] = ok ? load8(k + b * ks.b + h * ks.h + static_cast<int64_t>(my_key) * ks.s + 16 * s + 8 * hf) : zero8();
    vf[s] = ok ? load8(v + b * vs.b + h * vs.h + static_cast<int64_t>(my_key) * vs.s + 16 * s + 8 * hf) : zero8();
  }
  f32x16 dkacc[D / 32], dvacc[D / 32];
#pragma unroll
  for (int n = 0; n < D / 32; ++n) {
    dkacc[n] = zero16();
    dvacc[n] = zero16();
  }
  // register double buffer for the next query tile
  uint4 pf[NPF];
  float pl = 0.f, pd = 0.f;
  constexpr bool ROWC = D == 128;
  const float inv_sl2 = 1.f / scale_log2;
  // Q / dO tiles through buffer descriptors ending after row Sq - 1: rows past it load as zeros
  // (hardware range check; see KVPrefetch), 32-bit lane offsets computed once
  constexpr int PER = NPF / 2;  // chunks per thread per tensor (j < PER: Q, else dO)
  const uint32_t qstep = static_cast<uint32_t>(qs.s) * 2u, dstep = static_cast<uint32_t>(dos.s) * 2u;
  __amdgpu_buffer_rsrc_t qr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(qb), 0, static_cast<int>((Sq - 1) * qstep + 2u * D), 0x00020000);
  __amdgpu_buffer_rsrc_t dr = qr;
  auto set_head = [&](int hq) {
    qb = q + b * qs.b + hq * qs.h;
    dob = dO + b * dos.b + hq * dos.h;
    bh = static_cast<int64_t>(b) * H + hq;
    qr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(qb), 0,
                                           static_cast<int>((Sq - 1) * qstep + 2u * D), 0x00020000);
    dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(dob), 0,
                                           static_cast<int>((Sq - 1) * dstep + 2u * D), 0x00020000);
  };
  uint32_t pvo[NPF];
#pragma unroll
  for (int j = 0; j < NPF; ++j) {
    const int cc = threadIdx.x + 256 * (j % PER);
    pvo[j] = static_cast<uint32_t>(cc / CPR) * (j < PER ? qstep : dstep) + 2u * ((cc % CPR) * 8);
  }
  auto fetch = [&](int qt) {
    const uint32_t qo = static_cast<uint32_t>(qt) * qstep, dof = static_cast<uint32_t>(qt) * dstep;
#pragma unroll
    for (int j = 0; j < NPF; ++j)
      pf[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                            j < PER ? qr : dr, pvo[j] + (j < PER ? qo : dof), 0, 0));
    if (threadIdx.x < QT) {
      const int qi = qt + threadIdx.x;
      if constexpr (ROWC) {
        // staged as the accumulators' initial values (see the tile below): -LSE/scale_log2, -delta
        pl = qi < Sq ? -lse[bh * Sq + qi] * inv_sl2 : -INFINITY;
        pd = qi < Sq ? -delta[bh * Sq + qi] : 0.f;
      } else {
        pl = qi < Sq ? lse[bh * Sq + qi] : INFINITY;
        pd = qi < Sq ? delta[bh * Sq + qi] : 0.f;
      }
    }
  };
  const int tr_row = (r & 15) >> 2;
  const int tr_col = 16 * (r >> 4) + 4 * (r & 3);
  const int q_start = CAUSAL ? (k_blk / QT) * QT : 0;
  for (int g = 0; g < G; ++g) {
  set_head(h * G + g);
  if (q_start < Sq) fetch(q_start);
  for (int qt = q_start; qt < Sq; qt += QT) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      const int cc = threadIdx.x + 256 * (j % PER);
      const int row = cc / CPR, ch = cc % CPR;
      *reinterpret_cast<uint4*>((j >= PER ? dOs : Qs) + row * RS + ch * 8) = pf[j];
    }
    if (threadIdx.x < QT) {
      lse_s[threadIdx.x] = pl;
      del_s[threadIdx.x] = pd;
    }
    __syncthreads();
    if (qt + QT < Sq) fetch(qt + QT);
    // one 32-query MFMA sub-tile at LDS row offset 32*half (queries qs0 .. qs0+31)
    auto tile = [&](auto masked, const int half) {
      const int qs0 = qt + 32 * half;
      const uint16_t* Qh = Qs + 32 * half * RS;
      const uint16_t* dOh = dOs + 32 * half * RS;
      // ROWC (D = 128): row constants as the initial accumulators (guide: attention backward):
      // S' = Q K^T - LSE/scale_log2 and dP' = dO V^T - delta come out of the MFMA chains, so
      // p = exp2(S' * scale_log2) and dS = p * dP' need no per-element subtraction and no
      // registers for the constants (D = 128: +6%; D = 64: neutral, so off there --
      // profiles/round3_attention_bwd_ab.txt). This lane's 16 queries are 4 runs of 4 consecutive
      // rows: 16-B LDS reads straight into the accumulator registers.
      auto rows16 = [&](const float* base) {
        const f32x4* b4 = reinterpret_cast<const f32x4*>(base + 32 * half + 4 * hf);
        const f32x4 a0 = b4[0], a1 = b4[2], a2 = b4[4], a3 = b4[6];  // rows +0, +8, +16, +24
        return __builtin_shufflevector(__builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7),
                                       __builtin_shufflevector(a2, a3, 0, 1, 2, 3, 4, 5, 6, 7),
                                       0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
      };
      f32x16 sacc = ROWC ? rows16(lse_s) : zero16(), dpacc = ROWC ? rows16(del_s) : zero16();
      f32x16 lrow, drow;  // !ROWC: the same constants, subtracted per element below
      if constexpr (!ROWC) {
        lrow = rows16(lse_s);
        drow = rows16(del_s);
      }
      if constexpr (D == 64) {  // fragments preloaded (see the forward)
        bf16x8 qfr[D / 16], dofr[D / 16];
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          const int c = 16 * s + 8 * hf;
          qfr[s] = load8(Qh + r * RS + c);
          dofr[s] = load8(dOh + r * RS + c);
        }
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          sacc = mfma32(qfr[s], kf[s], sacc);
          dpacc = mfma32(dofr[s], vf[s], dpacc);
        }
      } else {
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          const int c = 16 * s + 8 * hf;
          sacc = mfma32(load8(Qh + r * RS + c), kf[s], sacc);
          dpacc = mfma32(load8(dOh + r * RS + c), vf[s], dpacc);
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = ROWC ? fast_exp2(sacc[i] * scale_log2) : fast_exp2(fmaf(sacc[i], scale_log2, -lrow[i]));
        if constexpr (decltype(masked)::value) {
          const int qi = qs0 + (i & 3) + 8 * (i >> 2) + 4 * hf;
          p = (qi >= Sq || my_key >= Sk || (CAUSAL && my_key > qi)) ? 0.f : p;
        }
        sacc[i] = p;
        dpacc[i] = ROWC ? p * dpacc[i] : p * (dpacc[i] - drow[i]);  // scale applied once to dK at the end
      }
      const bf16x8 p0 = pack8(sacc, 0), p1 = pack8(sacc, 8);
      const bf16x8 s0 = pack8(dpacc, 0), s1 = pack8(dpacc, 8);
#pragma unroll
      for (int n = 0; n < D / 32; ++n) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int off = (16 * s2 + 4 * hf + tr_row) * RS + 32 * n + tr_col;
          const int off8 = (16 * s2 + 4 * hf + tr_row + 8) * RS + 32 * n + tr_col;
          dvacc[n] = mfma32(cat8(tr_read(dOh + off), tr_read(dOh + off8)), s2 ? p1 : p0, dvacc[n]);
          dkacc[n] = mfma32(cat8(tr_read(Qh + off), tr_read(Qh + off8)), s2 ? s1 : s0, dkacc[n]);
        }
      }
    };
#pragma unroll
    for (int half = 0; half < QT / 32; ++half) {
      const int qs0 = qt + 32 * half;
      // wave-uniform: causal (keys after every query of the sub-tile), past Sq / Sk
      if (qs0 >= Sq || (CAUSAL && kw0 > qs0 + 31) || kw0 >= Sk) continue;
      // a key block straddling Sk only exists in the last workgroup
      if (D == 128 || (qs0 + 32 > Sq) || (kw0 + 32 > Sk) || (CAUSAL && kw0 + 31 > qs0))
        tile(std::true_type{}, half);
      else
        tile(std::false_type{}, half);
    }
  }
  }  // query heads of this K/V head
  store_rows<D>(dk + b * dks.b + h * dks.h + static_cast<int64_t>(my_key) * dks.s, dkacc, scale, hf, my_key < SkT);
  store_rows<D>(dv + b * dvs.b + h * dvs.h + static_cast<int64_t>(my_key) * dvs.s, dvacc, 1.f, hf, my_key < SkT);
}

// The dK/dV kernel with the Q / dO tiles (and the LSE / delta rows) through the 2-stage
// direct-to-LDS ring (KVDma): one flat (query head, query tile) sequence, one barrier per tile.
template <int D, bool CAUSAL, int QT, bool DMA = true>
__global__ __launch_bounds__(256, D == 64 ? 2 : 1) void attn_bwd_dkdv_dma_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
    const uint16_t* __restrict__ dO, const float* __restrict__ lse, const float* __restrict__ delta,
    uint16_t* __restrict__ dk, uint16_t* __restrict__ dv, int Sq, int Sk, int H, Strides qs,
    Strides ks, Strides vs, Strides dos, Strides dks, Strides dvs, float scale_log2, float scale,
    int order, const int* __restrict__ kvlen, int G) {
  constexpr int KB = 128;
  static_assert(QT == 32 || QT == 64, "query tile");
  constexpr int RS = D + kPad;
  constexpr int CPR = D / 8;                 // 16-byte chunks per row
  constexpr int NPF = 2 * QT * CPR / 256;    // prefetched chunks per thread (Q and dO tiles)
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  // register-staged: [QT][RS] Q | [QT][RS] dO | lse[QT] | delta[QT]; DMA: two such stages of
  // [QT][D] swizzled rows (see KVDma) -- QRS is the row stride either way
  constexpr int QRS = DMA ? D : RS;
  constexpr int STG = 2 * QT * QRS + 4 * QT;  // stage size in uint16 elements
  uint16_t* Qs = smem;
  uint16_t* dOs = Qs + QT * QRS;
  float* lse_s = reinterpret_cast<float*>(dOs + QT * QRS);
  float* del_s = lse_s + QT;
  const int lane = threadIdx.x & 63;
  // wave index in an SGPR: every per-wave condition below (causal extents, masking) is a
  // uniform branch instead of per-lane exec masking
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const Blk blk = xcd_block(order);
  const int b = blk.z, h = blk.y;
  const int SkT = Sk;  // rows of dK/dV to write (padded keys get zeros)
  // key padding: keys at or past kvlen[b] are masked like keys past Sk (>= 1 key kept)
  if (kvlen) Sk = min(Sk, max(kvlen[b], 1));
  const int k_blk = blk.x * KB;
  const int kw0 = k_blk + 32 * w;
  const int my_key = kw0 + r;
  // h is the K/V head (grid y runs over H / G of them); its G query heads h*G .. h*G+G-1 are swept
  // one after another below, dK / dV summing over all of them in the same registers
  const uint16_t* qb = q;
  const uint16_t* dob = dO;
  int64_t bh = 0;

  bf16x8 kf[D / 16], vf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const bool ok = my_key < Sk;
    kf[s] = ok ? load8(k + b * ks.b + h * ks.h + static_cast<int64_t>(my_key) * ks.s + 16 * s + 8 * hf) : zero8();
    vf[s] = ok ? load8(v + b * vs.b + h * vs.h + static_cast<int64_t>(my_key) * vs.s + 16 * s + 8 * hf) : zero8();
  }
  f32x16 dkacc[D / 32], dvacc[D / 32];
#pragma unroll
  for (int n = 0; n < D / 32; ++n) {
    dkacc[n] = zero16();
    dvacc[n] = zero16();
  }
  // register double buffer for the next query tile
  uint4 pf[NPF];
  float pl = 0.f, pd = 0.f;
  constexpr bool ROWC = D == 128;
  const float inv_sl2 = 1.f / scale_log2;
  // Q / dO tiles through buffer descriptors ending after row Sq - 1: rows past it load as zeros
  // (hardware range check; see KVPrefetch), 32-bit lane offsets computed once
  constexpr int PER = NPF / 2;  // chunks per thread per tensor (j < PER: Q, else dO)
  const uint32_t qstep = static_cast<uint32_t>(qs.s) * 2u, dstep = static_cast<uint32_t>(dos.s) * 2u;
  __amdgpu_buffer_rsrc_t qr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(qb), 0, static_cast<int>((Sq - 1) * qstep + 2u * D), 0x00020000);
  __amdgpu_buffer_rsrc_t dr = qr;
  auto set_head = [&](int hq) {
    qb = q + b * qs.b + hq * qs.h;
    dob = dO + b * dos.b + hq * dos.h;
    bh = static_cast<int64_t>(b) * H + hq;
    qr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(qb), 0,
                                           static_cast<int>((Sq - 1) * qstep + 2u * D), 0x00020000);
    dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(dob), 0,
                                           static_cast<int>((Sq - 1) * dstep + 2u * D), 0x00020000);
  };
  uint32_t pvo[NPF];
#pragma unroll
  for (int j = 0; j < NPF; ++j) {
    const int cc = threadIdx.x + 256 * (j % PER);
    pvo[j] = static_cast<uint32_t>(cc / CPR) * (j < PER ? qstep : dstep) + 2u * ((cc % CPR) * 8);
  }
  auto fetch = [&](int qt) {
    const uint32_t qo = static_cast<uint32_t>(qt) * qstep, dof = static_cast<uint32_t>(qt) * dstep;
#pragma unroll
    for (int j = 0; j < NPF; ++j)
      pf[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                            j < PER ? qr : dr, pvo[j] + (j < PER ? qo : dof), 0, 0));
    if (threadIdx.x < QT) {
      const int qi = qt + threadIdx.x;
      if constexpr (ROWC) {
        // staged as the accumulators' initial values (see the tile below): -LSE/scale_log2, -delta
        pl = qi < Sq ? -lse[bh * Sq + qi] * inv_sl2 : -INFINITY;
        pd = qi < Sq ? -delta[bh * Sq + qi] : 0.f;
      } else {
        pl = qi < Sq ? lse[bh * Sq + qi] : INFINITY;
        pd = qi < Sq ? delta[bh * Sq + qi] : 0.f;
      }
    }
  };
  const int tr_row = (r & 15) >> 2;
  const int tr_col = 16 * (r >> 4) + 4 * (r & 3);
  const int q_start = CAUSAL ? (k_blk / QT) * QT : 0;
  // the MFMA work on the staged query tile qt (Qs / dOs / lse_s / del_s)
  auto process = [&](const int qt) {
    // one 32-query MFMA sub-tile at LDS row offset 32*half (queries qs0 .. qs0+31)
    auto tile = [&](auto masked, const int half) {
      const int qs0 = qt + 32 * half;
      const uint16_t* Qh = Qs + 32 * half * QRS;
      const uint16_t* dOh = dOs + 32 * half * QRS;
      // ROWC (D = 128): row constants as the initial accumulators (guide: attention backward):
      // S' = Q K^T - LSE/scale_log2 and dP' = dO V^T - delta come out of the MFMA chains, so
      // p = exp2(S' * scale_log2) and dS = p * dP' need no per-element subtraction and no
      // registers for the constants (D = 128: +6%; D = 64: neutral, so off there --
      // profiles/round3_attention_bwd_ab.txt). This lane's 16 queries are 4 runs of 4 consecutive
      // rows: 16-B LDS reads straight into the accumulator registers.
      auto rows16 = [&](const float* base) {
        const f32x4* b4 = reinterpret_cast<const f32x4*>(base + 32 * half + 4 * hf);
        const f32x4 a0 = b4[0], a1 = b4[2], a2 = b4[4], a3 = b4[6];  // rows +0, +8, +16, +24
        return __builtin_shufflevector(__builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7),
                                       __builtin_shufflevector(a2, a3, 0, 1, 2, 3, 4, 5, 6, 7),
                                       0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
      };
      f32x16 sacc = ROWC ? rows16(lse_s) : zero16(), dpacc = ROWC ? rows16(del_s) : zero16();
      f32x16 lrow, drow;  // !ROWC: the same constants, subtracted per element below
      if constexpr (!ROWC) {
        lrow = rows16(lse_s);
        drow = rows16(del_s);
      }
      if constexpr (D == 64) {  // fragments preloaded (see the forward)
        bf16x8 qfr[D / 16], dofr[D / 16];
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          qfr[s] = load8(Qh + r * QRS + swz_off<D>(r, 2 * s + hf));
          dofr[s] = load8(dOh + r * QRS + swz_off<D>(r, 2 * s + hf));
        }
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          sacc = mfma32(qfr[s], kf[s], sacc);
          dpacc = mfma32(dofr[s], vf[s], dpacc);
        }
      } else {
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          sacc = mfma32(load8(Qh + r * QRS + swz_off<D>(r, 2 * s + hf)), kf[s], sacc);
          dpacc = mfma32(load8(dOh + r * QRS + swz_off<D>(r, 2 * s + hf)), vf[s], dpacc);
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = ROWC ? fast_exp2(sacc[i] * scale_log2) : fast_exp2(fmaf(sacc[i], scale_log2, -lrow[i]));
        if constexpr (decltype(masked)::value) {
          const int qi = qs0 + (i & 3) + 8 * (i >> 2) + 4 * hf;
          p = (qi >= Sq || my_key >= Sk || (CAUSAL && my_key > qi)) ? 0.f : p;
        }
        sacc[i] = p;
        dpacc[i] = ROWC ? p * dpacc[i] : p * (dpacc[i] - drow[i]);  // scale applied once to dK at the end
      }
      const bf16x8 p0 = pack8(sacc, 0), p1 = pack8(sacc, 8);
      const bf16x8 s0 = pack8(dpacc, 0), s1 = pack8(dpacc, 8);
#pragma unroll
      for (int n = 0; n < D / 32; ++n) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int off = (16 * s2 + 4 * hf + tr_row) * QRS + tr_off<D>(lane, n, false);
          const int off8 = (16 * s2 + 4 * hf + tr_row + 8) * QRS + tr_off<D>(lane, n, true);
          dvacc[n] = mfma32(cat8(tr_read(dOh + off), tr_read(dOh + off8)), s2 ? p1 : p0, dvacc[n]);
          dkacc[n] = mfma32(cat8(tr_read(Qh + off), tr_read(Qh + off8)), s2 ? s1 : s0, dkacc[n]);
        }
      }
    };
#pragma unroll
    for (int half = 0; half < QT / 32; ++half) {
      const int qs0 = qt + 32 * half;
      // wave-uniform: causal (keys after every query of the sub-tile), past Sq / Sk
      if (qs0 >= Sq || (CAUSAL && kw0 > qs0 + 31) || kw0 >= Sk) continue;
      // a key block straddling Sk only exists in the last workgroup
      if (D == 128 || (qs0 + 32 > Sq) || (kw0 + 32 > Sk) || (CAUSAL && kw0 + 31 > qs0))
        tile(std::true_type{}, half);
      else
        tile(std::false_type{}, half);
    }
  };
  if constexpr (DMA) {
    // one flat sequence of (query head, query tile) through the 2-stage ring
    const int tph = q_start < Sq ? (Sq - q_start + QT - 1) / QT : 0;  // tiles per query head
    const int ntiles = G * tph;
    KVDma<D, QT> dma;
    auto rows_of = [&](int hq, int qt) {  // this tile's -LSE/scale_log2, -delta (ROWC) or LSE, delta
      if (threadIdx.x < QT) {
        const int qi = qt + threadIdx.x;
        const int64_t bq = static_cast<int64_t>(b) * H + hq;
        if constexpr (ROWC) {
          pl = qi < Sq ? -lse[bq * Sq + qi] * inv_sl2 : -INFINITY;
          pd = qi < Sq ? -delta[bq * Sq + qi] : 0.f;
        } else {
          pl = qi < Sq ? lse[bq * Sq + qi] : INFINITY;
          pd = qi < Sq ? delta[bq * Sq + qi] : 0.f;
        }
      }
    };
    if (ntiles > 0) {
      dma.init(q + b * qs.b + (h * G) * qs.h, qs, dO + b * dos.b + (h * G) * dos.h, dos, Sq, w, lane);
      dma.issue(smem, smem + QT * D, q_start, w);
      rows_of(h * G, q_start);
    }
    int stage = 0, cur_g = 0;
    for (int t = 0; t < ntiles; ++t) {
      const int qt = q_start + (t % tph) * QT;
      Qs = smem + stage * STG;
      dOs = Qs + QT * D;
      lse_s = reinterpret_cast<float*>(dOs + QT * D);
      del_s = lse_s + QT;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of the tile landed
      if (threadIdx.x < QT) {
        lse_s[threadIdx.x] = pl;
        del_s[threadIdx.x] = pd;
      }
      __syncthreads();  // everyone's tile + row constants; the other stage is free
      if (t + 1 < ntiles) {
        const int g1 = (t + 1) / tph, qt1 = q_start + ((t + 1) % tph) * QT;
        if (g1 != cur_g) {
          cur_g = g1;
          dma.set_base(q + b * qs.b + (h * G + g1) * qs.h, dO + b * dos.b + (h * G + g1) * dos.h, Sq);
        }
        uint16_t* nq = smem + (stage ^ 1) * STG;
        dma.issue(nq, nq + QT * D, qt1, w);
        rows_of(h * G + g1, qt1);
      }
      process(qt);
      stage ^= 1;
    }
  }
  store_rows<D>(dk + b * dks.b + h * dks.h + static_cast<int64_t>(my_key) * dks.s, dkacc, scale, hf, my_key < SkT);
  store_rows<D>(dv + b * dvs.b + h * dvs.h + static_cast<int64_t>(my_key) * dvs.s, dvacc, 1.f, hf, my_key < SkT);
}

// workgroup order (see xcd_block): causal launches heaviest-first (2) -- fwd +12-38%, bwd
// +10-23% over XCD remap alone at S 1024-4096 (profiles/round3_attention_lpt_order.txt); full
// attention XCD-remapped (1).
int attn_order(bool causal) { return causal ? 2 : 1; }

size_t bwd_dkdv_lds(int D, int QT) {
  return 2 * static_cast<size_t>(QT) * (D + kPad) * 2 + 2 * static_cast<size_t>(QT) * sizeof(float);
}

// Production configuration, each choice measured on MI355X (the A/B switches that chose them were
// removed in round 6; their profiles stay):
//  * forward: 64-key tiles through the 2-stage direct-to-LDS ring (KVDma, +1.5-8 % causal, +3-5 %
//    full: profiles/round5_attention_dma_ring_ab.txt), score products of a sub-tile pair issued
//    before their softmaxes (PIPE: D64 +5-10 %, D128 +1-3.5 %: round3_attention_ab.txt,
//    round4_attention_knobs.txt); 128-key tiles measured slower (round4_attention_knobs.txt);
//  * dQ: D = 128 through the DMA ring (+2 %); D = 64 register-staged 64-key tiles (the ring -1.5 %);
//  * dK/dV: D = 128 through the DMA ring; D = 64 register-staged 64-query tiles (at 246 of 256
//    VGPRs the ring's swizzled offsets spill it).
template <int D, bool C>
void launch_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* o, float* lse,
                int B, int H, int Sq, int Sk, Strides qs, Strides ks, Strides vs, Strides os,
                float scale_log2, const int* kvlen, int G, hipStream_t st) {
  const dim3 grid((Sq + 127) / 128, H, B);
  constexpr int KT = 64;
  const size_t lds = 2 * 2 * static_cast<size_t>(KT) * D * 2;
  auto kern = attn_fwd_kernel<D, C, KT, true, true>;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, st, q, k, v, o, lse, Sq, Sk, H, qs, ks, vs, os,
                     scale_log2, attn_order(C), kvlen, G);
}

template <int D, bool C>
void launch_bwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, const uint16_t* o,
                const uint16_t* dO, const float* lse, float* delta, uint16_t* dq, uint16_t* dk,
                uint16_t* dv, int B, int H, int Sq, int Sk, Strides qs, Strides ks, Strides vs,
                Strides os, Strides dos, Strides dqs, Strides dks, Strides dvs, float scale_log2,
                float scale, const int* kvlen, int G, hipStream_t st) {
  auto dq_go = [&](auto kern, size_t l1) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(l1));
    hipLaunchKernelGGL(kern, dim3((Sq + 127) / 128, H, B), dim3(256), l1, st, q, k, v, o, dO, lse,
                       delta, dq, Sq, Sk, H, qs, ks, vs, os, dos, dqs, scale_log2, scale, attn_order(C), kvlen, G);
  };
  if constexpr (D == 128) {
    dq_go(attn_bwd_dq_kernel<D, C, 64, false, true>, 2 * 2 * static_cast<size_t>(64) * D * 2);
    const size_t l2 = 2 * (2 * static_cast<size_t>(64) * D * 2 + 2 * 64 * sizeof(float));
    auto kern = attn_bwd_dkdv_dma_kernel<D, C, 64>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(l2));
    hipLaunchKernelGGL(kern, dim3((Sk + 127) / 128, H / G, B), dim3(256), l2, st, q, k, v, dO, lse,
                       delta, dk, dv, Sq, Sk, H, qs, ks, vs, dos, dks, dvs, scale_log2, scale,
                       attn_order(C), kvlen, G);
  } else {
    dq_go(attn_bwd_dq_kernel<D, C, 64, false>, 2 * static_cast<size_t>(64) * (D + kPad) * 2);
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, C, 64>), dim3((Sk + 127) / 128, H / G, B), dim3(256),
                       bwd_dkdv_lds(D, 64), st, q, k, v, dO, lse, delta, dk, dv, Sq, Sk, H, qs, ks,
                       vs, dos, dks, dvs, scale_log2, scale, attn_order(C), kvlen, G);
  }
}

}  // namespace

void attention_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H,
                   int Sq, int Sk, int D, const int64_t* qs, const int64_t* ks, const int64_t* vs,
                   const int64_t* os, float scale, bool causal, const int* kvlen, int G,
                   hipStream_t st) {
  const float sl2 = scale * 1.4426950408889634f;
  Strides a{qs[0], qs[1], qs[2]}, bb{ks[0], ks[1], ks[2]}, c{vs[0], vs[1], vs[2]}, d{os[0], os[1], os[2]};
  auto Q = static_cast<const uint16_t*>(q);
  auto K = static_cast<const uint16_t*>(k);
  auto V = static_cast<const uint16_t*>(v);
  auto O = static_cast<uint16_t*>(o);
  if (D == 64) {
    if (causal) launch_fwd<64, true>(Q, K, V, O, lse, B, H, Sq, Sk, a, bb, c, d, sl2, kvlen, G, st);
    else launch_fwd<64, false>(Q, K, V, O, lse, B, H, Sq, Sk, a, bb, c, d, sl2, kvlen, G, st);
  } else {
    if (causal) launch_fwd<128, true>(Q, K, V, O, lse, B, H, Sq, Sk, a, bb, c, d, sl2, kvlen, G, st);
    else launch_fwd<128, false>(Q, K, V, O, lse, B, H, Sq, Sk, a, bb, c, d, sl2, kvlen, G, st);
  }
}

void attention_bwd(const void* q, const void* k, const void* v, const void* o, const void* dO,
                   const float* lse, float* delta, float* dq_acc, void* dq, void* dk, void* dv,
                   int B, int H, int Sq, int Sk, int D, const int64_t* st_q, const int64_t* st_k,
                   const int64_t* st_v, const int64_t* st_o, const int64_t* st_do,
                   const int64_t* st_dq, const int64_t* st_dk, const int64_t* st_dv, float scale,
                   bool causal, const int* kvlen, int G, hipStream_t stream) {
  const float sl2 = scale * 1.4426950408889634f;
  auto S = [](const int64_t* p) { return Strides{p[0], p[1], p[2]}; };
  auto c16 = [](const void* p) { return static_cast<const uint16_t*>(p); };
  auto m16 = [](void* p) { return static_cast<uint16_t*>(p); };
  if (D == 64) {
    if (causal) launch_bwd<64, true>(c16(q), c16(k), c16(v), c16(o), c16(dO), lse, delta, m16(dq), m16(dk), m16(dv), B, H, Sq, Sk, S(st_q), S(st_k), S(st_v), S(st_o), S(st_do), S(st_dq), S(st_dk), S(st_dv), sl2, scale, kvlen, G, stream);
    else launch_bwd<64, false>(c16(q), c16(k), c16(v), c16(o), c16(dO), lse, delta, m16(dq), m16(dk), m16(dv), B, H, Sq, Sk, S(st_q), S(st_k), S(st_v), S(st_o), S(st_do), S(st_dq), S(st_dk), S(st_dv), sl2, scale, kvlen, G, stream);
  } else {
    if (causal) launch_bwd<128, true>(c16(q), c16(k), c16(v), c16(o), c16(dO), lse, delta, m16(dq), m16(dk), m16(dv), B, H, Sq, Sk, S(st_q), S(st_k), S(st_v), S(st_o), S(st_do), S(st_dq), S(st_dk), S(st_dv), sl2, scale, kvlen, G, stream);
    else launch_bwd<128, false>(c16(q), c16(k), c16(v), c16(o), c16(dO), lse, delta, m16(dq), m16(dk), m16(dv), B, H, Sq, Sk, S(st_q), S(st_k), S(st_v), S(st_o), S(st_do), S(st_dq), S(st_dk), S(st_dv), sl2, scale, kvlen, G, stream);
  }
}

}  // namespace dca
