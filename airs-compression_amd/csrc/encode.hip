// encode.hip -- MI355X (gfx950) kernels for the AIRSPACE encode hot path.
//
// Replaces the reference's per-sample loop lib/compress/cmp.c:296-312
// (predictor -> ZigZag -> Golomb -> big-endian bit packing) with one
// data-parallel pass over HBM:
//
//   segment  = 4096 consecutive samples of one frame = one 256-thread workgroup
//              (16 samples per lane, contiguous)
//   1. ticket      workgroups take segments in dispatch order (atomic ticket),
//                  so a segment only ever waits on segments already running
//   2. load        16 samples / lane straight from HBM (dwordx4), model too
//   3. code        residual (NONE / DIFF / MODEL), ZigZag, Golomb codeword and
//                  length per sample, in registers
//   4. scan        wave shuffle scan + LDS across the 4 waves -> each lane's
//                  bit offset inside the segment and the segment's bit total
//   5. publish     segment total ("aggregate") to a tagged 64-bit granule
//   6. pack        each lane ORs its codewords into an LDS image of the
//                  segment's bit stream, aligned at bit 0
//   7. look-back   wave 0 sums predecessor granules (decoupled look-back,
//                  64 granules per step) -> the segment's frame bit offset P
//   8. store       the LDS image is funnel-shifted by P mod 32 on the way out
//                  (v_alignbit) and written as big-endian dwords; the word
//                  shared with the predecessor is completed with the
//                  predecessor's published last 32 bits ("tail" granule)
//   9. epilogue    the frame's last segment writes the header (with the final
//                  size), the zero-padded last bytes, the checksum and status
//
// Nothing is MFMA-shaped here: this is integer bit work bound by HBM reads.
// Cross-workgroup data moves only through 8-byte granules that carry their own
// epoch tag (written with one agent-scope atomic store, polled with
// agent-scope atomic loads), so no fences are needed (MI355X_MICROARCH.md,
// "R2" granule hand-off).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "airs_dev.h"

#include "enc_common.h"
#include "enc_kernel.h"

namespace airs {

// ---------------------------------------------------------------------
// Multi-level integer wavelet transform (reference preprocess.c:140-221,
// iwt_init :321-353): levels with stride s = 1, 2, 4, ... < n, each a lifting
// step in place: first every odd coefficient (index s mod 2s) from its even
// neighbours, then every even one from the new odd neighbours.  All values
// are int16 with the reference's int32 intermediates and int16 wrap.  The
// coefficients go to the frame's work buffer, where the encoder reads them as
// its residuals (iwt_process :366-371).
// ---------------------------------------------------------------------
__device__ __forceinline__ int16_t iwt_odd(int32_t c, int32_t l, int32_t r)
{
	return (int16_t)(c - (int16_t)((l + r) >> 1)); // iwt_odd_coefficient :67-70
}

__device__ __forceinline__ int16_t iwt_even(int32_t c, int32_t l, int32_t r)
{
	return (int16_t)(c + (int16_t)((l + r) >> 2)); // iwt_even_coefficient :96-100
}

__device__ __forceinline__ int16_t iwt_edge(int32_t c, int32_t nb)
{
	return (int16_t)(c + (int16_t)(nb >> 1)); // iwt_edge_even_coefficient :112-115
}

// odd coefficients of level s for t = t0, t0 + dt, ... (index i = s + 2 s t)
template <typename P>
__device__ __forceinline__ void iwt_odds(P y, uint32_t n, uint32_t s, uint32_t t0, uint32_t dt)
{
	for (uint32_t t = t0;; t += dt) {
		const uint64_t i = (uint64_t)s + 2ull * s * t;
		if (i >= n)
			break;
		// the last odd coefficient has no right neighbour (:81-84)
		y[i] = i + s < n ? iwt_odd(y[i], y[i - s], y[i + s]) : (int16_t)(y[i] - y[i - s]);
	}
}

// even coefficients of level s (index i = 2 s t); needs the level's odds
template <typename P>
__device__ __forceinline__ void iwt_evens(P y, uint32_t n, uint32_t s, uint32_t t0, uint32_t dt)
{
	for (uint32_t t = t0;; t += dt) {
		const uint64_t i = 2ull * s * t;
		if (i >= n)
			break;
		if (i == 0)
			y[0] = iwt_edge(y[0], y[s]);
		else if (i + s < n)
			y[i] = iwt_even(y[i], y[i - s], y[i + s]);
		else
			y[i] = iwt_edge(y[i], y[i - s]);
	}
}

struct IwtArgs {
	const uint8_t *src;
	uint64_t src_stride;
	uint8_t *coef; // work buffers: frame f's at coef + (f / coef_div) * coef_stride, or coef_ptrs[j]
	uint64_t coef_stride;
	const uint64_t *coef_ptrs;
	const uint32_t *frame_list;
	uint32_t frame_add, frame_mul, coef_div;
	uint32_t n;
	int16_t *heads; // two-phase kernels: launch frame j's block heads at heads + j * n / 64
};

__device__ __forceinline__ int16_t *iwt_frame_coef(const IwtArgs &a, uint32_t j, uint32_t *frame)
{
	*frame = a.frame_list ? a.frame_list[j] : a.frame_add + j * a.frame_mul;
	return reinterpret_cast<int16_t *>(a.coef_ptrs ? reinterpret_cast<uint8_t *>(a.coef_ptrs[j])
						       : a.coef + (uint64_t)(*frame / a.coef_div) * a.coef_stride);
}

template <int W>
__device__ __forceinline__ int16_t iwt_sample(const uint8_t *fsrc, uint32_t i)
{
	return W == 2 ? reinterpret_cast<const int16_t *>(fsrc)[i]
		      : (int16_t)(reinterpret_cast<const uint32_t *>(fsrc)[i] & 0xFFFFu); // sample_read_i16
}

// whole frame in LDS (n <= AIRS_IWT_LDS_MAX): one 1024-thread workgroup per frame
#define AIRS_IWT_LDS_MAX 65536u
// LDS view of a frame with a bank swizzle: element i lives in 32-bit word
// w ^ ((w >> 5) & 31), w = i / 2, so the stride-2s accesses of a level spread
// over the LDS banks instead of piling onto one
struct IwtLds {
	int16_t *base;
	__device__ __forceinline__ int16_t &operator[](uint64_t i) const
	{
		const uint32_t w = (uint32_t)i >> 1;
		return base[2u * (w ^ ((w >> 5) & 31u)) + ((uint32_t)i & 1u)];
	}
};

// one phase of level s in LDS: the odd (ODD) or even coefficients, four items
// per thread per round with all their operands loaded before any store (a
// phase never reads what it writes, except each item its own slot)
template <bool ODD, uint32_t NT = 1024u>
__device__ __forceinline__ void iwt_phase_lds(const IwtLds &y, uint32_t n, uint32_t s, uint32_t tid)
{
	const uint32_t cnt = ODD ? (n > s ? (n - s + 2u * s - 1u) / (2u * s) : 0u) : (n + 2u * s - 1u) / (2u * s);
	for (uint32_t b0 = 0; b0 < cnt; b0 += 4u * NT) {
		int32_t c[4], l[4], r[4];
		uint32_t idx[4];
		// neighbour indices clamped into the frame (a missing neighbour reads
		// the item itself and is not used), so every load is unconditional
#pragma unroll
		for (uint32_t u = 0; u < 4; u++) {
			const uint32_t t = min(b0 + u * NT + tid, cnt - 1u);
			const uint32_t i = ODD ? s + 2u * s * t : 2u * s * t;
			idx[u] = i;
			c[u] = y[i];
			l[u] = y[i >= s ? i - s : i];
			r[u] = y[i + s < n ? i + s : i];
		}
#pragma unroll
		for (uint32_t u = 0; u < 4; u++) {
			const uint32_t i = idx[u];
			int16_t v;
			if (ODD)
				v = i + s < n ? iwt_odd(c[u], l[u], r[u]) : (int16_t)(c[u] - l[u]);
			else
				v = i == 0 ? iwt_edge(c[u], r[u]) : i + s < n ? iwt_even(c[u], l[u], r[u]) : iwt_edge(c[u], l[u]);
			if (b0 + u * NT + tid < cnt)
				y[i] = v;
		}
	}
}

template <int W>
__global__ __launch_bounds__(1024) void iwt_frame_kernel(IwtArgs a)
{
	extern __shared__ int16_t L_iwt[];
	uint32_t frame;
	int16_t *coef = iwt_frame_coef(a, blockIdx.x, &frame);
	if (frame == AIRS_NO_FRAME) // a hole of the launch's frame list (device exact mode)
		return;
	const uint8_t *fsrc = a.src + (uint64_t)frame * a.src_stride;
	const uint32_t n = a.n, tid = threadIdx.x;
	const IwtLds y{L_iwt};
	// samples -> LDS: 16-byte loads when the frame is 16-byte aligned
	uint32_t done = 0;
	if (((uintptr_t)fsrc & 15u) == 0) {
		constexpr uint32_t PER = 16u / W; // samples per 16-byte load
		const uint32_t nq = n / PER;
		for (uint32_t q = tid; q < nq; q += 1024u) {
			const uint4 v = reinterpret_cast<const uint4 *>(fsrc)[q];
			const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
			for (uint32_t e = 0; e < 4; e++) {
				if (W == 2) {
					y[PER * q + 2u * e] = (int16_t)(vw[e] & 0xFFFFu);
					y[PER * q + 2u * e + 1u] = (int16_t)(vw[e] >> 16);
				} else {
					y[PER * q + e] = (int16_t)(vw[e] & 0xFFFFu);
				}
			}
		}
		done = nq * PER;
	}
	for (uint32_t i = done + tid; i < n; i += 1024u)
		y[i] = iwt_sample<W>(fsrc, i);
	__syncthreads();
#ifndef AIRS_IWT_ABL
#define AIRS_IWT_ABL 0
#endif
	for (uint32_t s = 1; s < (AIRS_IWT_ABL ? 0u : n); s <<= 1) {
		iwt_phase_lds<true>(y, n, s, tid);
		__syncthreads();
		iwt_phase_lds<false>(y, n, s, tid);
		__syncthreads();
	}
	// LDS -> work buffer: two coefficients per 32-bit store when aligned
	if (((uintptr_t)coef & 3u) == 0) {
		uint32_t *c32 = reinterpret_cast<uint32_t *>(coef);
		for (uint32_t q = tid; q < n / 2u; q += 1024u)
			c32[q] = (uint32_t)(uint16_t)y[2u * q] | ((uint32_t)(uint16_t)y[2u * q + 1u] << 16);
		if ((n & 1u) && tid == 0)
			coef[n - 1u] = y[n - 1u];
	} else {
		for (uint32_t i = tid; i < n; i += 1024u)
			coef[i] = y[i];
	}
}

// Frames of 64 k samples (n a multiple of 64, n <= 65536): thread t holds
// samples [64t, 64t + 64) in registers and runs the six levels s = 1 .. 32
// there; per level it needs the next block's first sample (odd phase) and
// the previous block's last odd coefficient (even phase), swapped through
// LDS.  The remaining levels (strides 64, 128, ...) act on the n / 64 block
// heads, which the LDS phases handle as a frame of their own.
template <int W>
__global__ __launch_bounds__(1024) void iwt_block_kernel(IwtArgs a)
{
	__shared__ int16_t h_first[1024], h_odd[1024], heads[1024 + 64];
	uint32_t frame;
	int16_t *coef = iwt_frame_coef(a, blockIdx.x, &frame);
	if (frame == AIRS_NO_FRAME) // a hole of the launch's frame list (device exact mode)
		return;
	const uint8_t *fsrc = a.src + (uint64_t)frame * a.src_stride;
	const uint32_t n = a.n, nb = n / 64u, t = threadIdx.x;
	const bool act = t < nb, last = t + 1u == nb;
	int32_t x[64];
	if (act) {
		const uint4 *p = reinterpret_cast<const uint4 *>(fsrc + (size_t)t * 64u * W);
#pragma unroll
		for (uint32_t q = 0; q < 64u * W / 16u; q++) {
			const uint4 v = p[q];
			const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
			for (uint32_t e = 0; e < 4; e++) {
				if (W == 2) {
					x[8 * q + 2 * e] = (int16_t)(vw[e] & 0xFFFFu);
					x[8 * q + 2 * e + 1] = (int16_t)(vw[e] >> 16);
				} else {
					x[4 * q + e] = (int16_t)(vw[e] & 0xFFFFu);
				}
			}
		}
	}
#pragma unroll
	for (uint32_t s = 1; s < 64u; s <<= 1) {
		if (act)
			h_first[t] = (int16_t)x[0];
		__syncthreads();
		const int32_t rh = act && !last ? h_first[t + 1u] : 0;
#pragma unroll
		for (uint32_t k = s; k < 64u; k += 2u * s) {
			if (k + s < 64u)
				x[k] = iwt_odd(x[k], x[k - s], x[k + s]);
			else // the block's last odd: its right neighbour is the next block's head
				x[k] = last ? (int16_t)(x[k] - x[k - s]) : iwt_odd(x[k], x[k - s], rh);
		}
		if (act)
			h_odd[t] = (int16_t)x[64u - s];
		__syncthreads();
		const int32_t lh = act && t ? h_odd[t - 1u] : 0;
		x[0] = t ? iwt_even(x[0], lh, x[s]) : iwt_edge(x[0], x[s]);
#pragma unroll
		for (uint32_t k = 2u * s; k < 64u; k += 2u * s)
			x[k] = iwt_even(x[k], x[k - s], x[k + s]);
	}
	// strides 64, 128, ...: the block heads as a frame of nb samples
	const IwtLds y{heads};
	if (act)
		y[t] = (int16_t)x[0];
	__syncthreads();
	for (uint32_t s = 1; s < nb; s <<= 1) {
		iwt_phase_lds<true>(y, nb, s, t);
		__syncthreads();
		iwt_phase_lds<false>(y, nb, s, t);
		__syncthreads();
	}
	if (act) {
		x[0] = y[t];
		uint4 *o = reinterpret_cast<uint4 *>(coef + (size_t)t * 64u);
#pragma unroll
		for (uint32_t q = 0; q < 8u; q++)
			o[q] = make_uint4((uint32_t)(uint16_t)x[8 * q] | ((uint32_t)(uint16_t)x[8 * q + 1] << 16),
					  (uint32_t)(uint16_t)x[8 * q + 2] | ((uint32_t)(uint16_t)x[8 * q + 3] << 16),
					  (uint32_t)(uint16_t)x[8 * q + 4] | ((uint32_t)(uint16_t)x[8 * q + 5] << 16),
					  (uint32_t)(uint16_t)x[8 * q + 6] | ((uint32_t)(uint16_t)x[8 * q + 7] << 16));
	}
}

// Frames of any size with n a multiple of 64 (n >= 128), in two launches.
// Phase A: a 256-thread workgroup takes IWT_RB = 252 consecutive 64-sample
// blocks of a frame plus two halo blocks on each side (the dependency cone of
// six levels is under 128 samples), runs levels s = 1 .. 32 in registers as
// iwt_block_kernel does, and writes its real blocks (their heads still at
// level 6).  Phase B: one workgroup per frame runs the levels s >= 64 on the
// n / 64 heads in LDS and writes them back.
#define IWT_RB 252u
template <int W>
__global__ __launch_bounds__(256) void iwt_blocks_a_kernel(IwtArgs a, uint32_t wg_per_frame)
{
	__shared__ int16_t h_first[256], h_odd[256];
	const uint32_t j = blockIdx.x / wg_per_frame, part = blockIdx.x - j * wg_per_frame;
	uint32_t frame;
	int16_t *coef = iwt_frame_coef(a, j, &frame);
	if (frame == AIRS_NO_FRAME) // a hole of the launch's frame list (device exact mode)
		return;
	const uint8_t *fsrc = a.src + (uint64_t)frame * a.src_stride;
	const uint32_t nb = a.n / 64u, t = threadIdx.x;
	const int32_t gb = (int32_t)(part * IWT_RB + t) - 2; // global block of this thread
	const bool act = gb >= 0 && gb < (int32_t)nb;
	const bool first = gb == 0, last = gb + 1 == (int32_t)nb;
	int32_t x[64];
	if (act) {
		const uint4 *p = reinterpret_cast<const uint4 *>(fsrc + (size_t)gb * 64u * W);
#pragma unroll
		for (uint32_t q = 0; q < 64u * W / 16u; q++) {
			const uint4 v = p[q];
			const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
			for (uint32_t e = 0; e < 4; e++) {
				if (W == 2) {
					x[8 * q + 2 * e] = (int16_t)(vw[e] & 0xFFFFu);
					x[8 * q + 2 * e + 1] = (int16_t)(vw[e] >> 16);
				} else {
					x[4 * q + e] = (int16_t)(vw[e] & 0xFFFFu);
				}
			}
		}
	} else {
#pragma unroll
		for (uint32_t k = 0; k < 64u; k++)
			x[k] = 0;
	}
#pragma unroll
	for (uint32_t s = 1; s < 64u; s <<= 1) {
		h_first[t] = (int16_t)x[0];
		__syncthreads();
		const int32_t rh = t + 1u < 256u ? h_first[t + 1u] : 0;
#pragma unroll
		for (uint32_t k = s; k < 64u; k += 2u * s) {
			if (k + s < 64u)
				x[k] = iwt_odd(x[k], x[k - s], x[k + s]);
			else
				x[k] = last ? (int16_t)(x[k] - x[k - s]) : iwt_odd(x[k], x[k - s], rh);
		}
		h_odd[t] = (int16_t)x[64u - s];
		__syncthreads();
		const int32_t lh = t ? h_odd[t - 1u] : 0;
		x[0] = first ? iwt_edge(x[0], x[s]) : iwt_even(x[0], lh, x[s]);
#pragma unroll
		for (uint32_t k = 2u * s; k < 64u; k += 2u * s)
			x[k] = iwt_even(x[k], x[k - s], x[k + s]);
	}
	if (act && t >= 2u && t < 2u + IWT_RB) {
		a.heads[(size_t)j * nb + gb] = (int16_t)x[0];
		uint4 *o = reinterpret_cast<uint4 *>(coef + (size_t)gb * 64u);
#pragma unroll
		for (uint32_t q = 0; q < 8u; q++)
			o[q] = make_uint4((uint32_t)(uint16_t)x[8 * q] | ((uint32_t)(uint16_t)x[8 * q + 1] << 16),
					  (uint32_t)(uint16_t)x[8 * q + 2] | ((uint32_t)(uint16_t)x[8 * q + 3] << 16),
					  (uint32_t)(uint16_t)x[8 * q + 4] | ((uint32_t)(uint16_t)x[8 * q + 5] << 16),
					  (uint32_t)(uint16_t)x[8 * q + 6] | ((uint32_t)(uint16_t)x[8 * q + 7] << 16));
	}
}

// one wave per frame: the heads are few (n / 64), and a one-wave workgroup
// pays nothing for its barriers
__global__ __launch_bounds__(64) void iwt_heads_b_kernel(IwtArgs a)
{
	extern __shared__ int16_t L_heads[];
	uint32_t frame;
	int16_t *coef = iwt_frame_coef(a, blockIdx.x, &frame);
	if (frame == AIRS_NO_FRAME) // a hole of the launch's frame list (device exact mode)
		return;
	const uint32_t nb = a.n / 64u, t = threadIdx.x;
	const IwtLds y{L_heads};
	const int16_t *hd = a.heads + (size_t)blockIdx.x * nb;
	for (uint32_t i = t; i < nb; i += 64u)
		y[i] = hd[i];
	__syncthreads();
	for (uint32_t s = 1; s < nb; s <<= 1) {
		iwt_phase_lds<true, 64u>(y, nb, s, t);
		__syncthreads();
		iwt_phase_lds<false, 64u>(y, nb, s, t);
		__syncthreads();
	}
	for (uint32_t i = t; i < nb; i += 64u)
		coef[(size_t)i * 64u] = y[i];
}

// larger frames: samples -> work buffer, then two launches per level
template <int W>
__global__ __launch_bounds__(256) void iwt_copy_kernel(IwtArgs a)
{
	uint32_t frame;
	int16_t *coef = iwt_frame_coef(a, blockIdx.y, &frame);
	if (frame == AIRS_NO_FRAME) // a hole of the launch's frame list (device exact mode)
		return;
	const uint8_t *fsrc = a.src + (uint64_t)frame * a.src_stride;
	for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < a.n; i += gridDim.x * 256u)
		coef[i] = iwt_sample<W>(fsrc, i);
}

__global__ __launch_bounds__(256) void iwt_level_kernel(IwtArgs a, uint32_t s, uint32_t evens)
{
	uint32_t frame;
	int16_t *coef = iwt_frame_coef(a, blockIdx.y, &frame);
	if (frame == AIRS_NO_FRAME) // a hole of the launch's frame list (device exact mode)
		return;
	const uint32_t t0 = blockIdx.x * 256u + threadIdx.x, dt = gridDim.x * 256u;
	if (evens)
		iwt_evens(coef, a.n, s, t0, dt);
	else
		iwt_odds(coef, a.n, s, t0, dt);
}

// ---------------------------------------------------------------------
// XXH32 per frame over big-endian 16-bit samples (reference header.c:137-163).
// The four accumulators of a frame run in four lanes; each stripe is 8
// samples = 16 bytes, lane q consumes bytes 4q..4q+3 of every stripe.
// ---------------------------------------------------------------------
#define XP1 2654435761u
#define XP2 2246822519u
#define XP3 3266489917u
#define XP4 668265263u
#define XP5 374761393u

__device__ __forceinline__ uint32_t rotl32(uint32_t x, uint32_t r)
{
	return (x << r) | (x >> (32u - r));
}

template <int W>
__device__ __forceinline__ uint32_t sample_at(const uint8_t *f, uint32_t i)
{
	return W == 2 ? (uint32_t)reinterpret_cast<const uint16_t *>(f)[i]
		      : reinterpret_cast<const uint32_t *>(f)[i] & 0xFFFFu;
}

// little-endian read of the BE byte image: bytes (hi0, lo0, hi1, lo1)
__device__ __forceinline__ uint32_t be_pair(uint32_t s0, uint32_t s1)
{
	return ((s0 >> 8) & 0xFFu) | ((s0 & 0xFFu) << 8) | (((s1 >> 8) & 0xFFu) << 16) | ((s1 & 0xFFu) << 24);
}

// one XXH32 round with the input's P2 product already formed: add, rotate,
// multiply as three dependent instructions (the compiler would fuse the add
// into a 64-bit v_mad_u64_u32, whose latency is longer)
__device__ __forceinline__ uint32_t xxh_round_pre(uint32_t acc, uint32_t yp2)
{
	asm volatile("v_add_u32 %0, %0, %1\n\tv_alignbit_b32 %0, %0, %0, 19\n\tv_mul_lo_u32 %0, %0, %2"
		     : "+v"(acc)
		     : "v"(yp2), "s"(XP1));
	return acc;
}

// XXH32 in two launches (the default): ck_pre_kernel forms every stripe's
// four inputs x P2 (the big-endian words of the samples, multiplied off the
// chain) into a scratch buffer with all the parallelism of the frame;
// ck_chain_kernel then runs only the 64 serial chains of 16 frames per wave,
// reading its inputs 128 rounds ahead.  Y is laid out for the chain wave:
// per group of 16 frames, for every 4 rounds, 64 chains x 16 bytes
// (chain = 4 (frame % 16) + accumulator), so one 16-byte load per lane reads
// 1 KiB contiguous.  S4 = stripes rounded up to 4.
template <int W>
__global__ __launch_bounds__(256) void ck_pre_kernel(const uint8_t *src, uint64_t stride, uint32_t n,
						     uint32_t num_frames, const uint32_t *frame_list, uint32_t S4,
						     uint32_t *Y)
{
	// a workgroup covers 16 frames x 16 round quads, frame fastest: the 64
	// lanes of a wave write 4 KiB of Y contiguous (their four stores fill it)
	const uint32_t stripes = n / 8u;
	const uint32_t lf = blockIdx.x * 16u + (threadIdx.x & 15u);
	if (lf >= num_frames)
		return;
	const uint32_t frame = frame_list ? frame_list[lf] : lf;
	const uint8_t *f = src + (uint64_t)frame * stride;
	// rounds 4 r4 .. 4 r4 + 3 (grid-stride: gridDim.y is capped)
	for (uint32_t r4 = blockIdx.y * 16u + (threadIdx.x >> 4); 4u * r4 < stripes; r4 += gridDim.y * 16u) {
		uint32_t y[4][4]; // [round][accumulator]
		if (4u * r4 + 4u <= stripes && ((uintptr_t)f & 15u) == 0u) {
#pragma unroll
			for (uint32_t t = 0; t < 4u; t++) {
				const uint32_t r = 4u * r4 + t;
				if (W == 2) {
					const uint4 v = reinterpret_cast<const uint4 *>(f)[r];
					y[t][0] = __builtin_amdgcn_perm(v.x, v.x, 0x02030001u);
					y[t][1] = __builtin_amdgcn_perm(v.y, v.y, 0x02030001u);
					y[t][2] = __builtin_amdgcn_perm(v.z, v.z, 0x02030001u);
					y[t][3] = __builtin_amdgcn_perm(v.w, v.w, 0x02030001u);
				} else {
					const uint4 a = reinterpret_cast<const uint4 *>(f)[2u * r];
					const uint4 b = reinterpret_cast<const uint4 *>(f)[2u * r + 1u];
					y[t][0] = be_pair(a.x & 0xFFFFu, a.y & 0xFFFFu);
					y[t][1] = be_pair(a.z & 0xFFFFu, a.w & 0xFFFFu);
					y[t][2] = be_pair(b.x & 0xFFFFu, b.y & 0xFFFFu);
					y[t][3] = be_pair(b.z & 0xFFFFu, b.w & 0xFFFFu);
				}
			}
		} else {
#pragma unroll
			for (uint32_t t = 0; t < 4u; t++) {
				const uint32_t r = 4u * r4 + t;
#pragma unroll
				for (uint32_t q = 0; q < 4u; q++)
					y[t][q] = r < stripes ? be_pair(sample_at<W>(f, 8u * r + 2u * q),
								     sample_at<W>(f, 8u * r + 2u * q + 1u))
							   : 0u;
			}
		}
		uint4 *G = reinterpret_cast<uint4 *>(Y + (uint64_t)(lf >> 4) * 64u * S4) + (uint64_t)r4 * 64u + (lf & 15u) * 4u;
#pragma unroll
		for (uint32_t q = 0; q < 4u; q++)
			G[q] = make_uint4(y[0][q] * XP2, y[1][q] * XP2, y[2][q] * XP2, y[3][q] * XP2);
	}
}

template <int W>
__global__ __launch_bounds__(64) void ck_chain_kernel(const uint8_t *src, uint64_t stride, uint32_t n,
						      uint32_t num_frames, const uint32_t *frame_list, uint32_t S4,
						      const uint32_t *Y, uint32_t *out)
{
	const uint32_t lane = threadIdx.x, q = lane & 3u;
	const uint32_t lf = blockIdx.x * 16u + (lane >> 2);
	const bool valid = lf < num_frames;
	const uint32_t len = 2u * n;
	const uint32_t stripes = len >= 16u ? n / 8u : 0u;
	const uint32_t seed = 419764627u;
	uint32_t acc = q == 0 ? seed + XP1 + XP2 : q == 1 ? seed + XP2 : q == 2 ? seed : seed - XP1;
	// this lane's chain: 16 bytes (4 rounds) every 1 KiB of its group
	const uint4 *P = reinterpret_cast<const uint4 *>(Y + (uint64_t)blockIdx.x * 64u * S4) + lane;
	// batches of 128 rounds (32 x 16 bytes per lane), the next batch loading
	// while this one runs
	constexpr uint32_t B = 32u;
	const uint32_t nb = stripes / (4u * B);
	uint4 cur[B], nxt[B];
	if (nb) {
#pragma unroll
		for (uint32_t u = 0; u < B; u++)
			cur[u] = P[64u * u];
	}
	for (uint32_t b = 0; b < nb; b++) {
		const uint32_t nbase = (b + 1u < nb ? b + 1u : b) * B;
#pragma unroll
		for (uint32_t u = 0; u < B; u++)
			nxt[u] = P[64u * (nbase + u)];
#pragma unroll
		for (uint32_t u = 0; u < B; u++) {
			acc = xxh_round_pre(acc, cur[u].x);
			acc = xxh_round_pre(acc, cur[u].y);
			acc = xxh_round_pre(acc, cur[u].z);
			acc = xxh_round_pre(acc, cur[u].w);
		}
#pragma unroll
		for (uint32_t u = 0; u < B; u++)
			cur[u] = nxt[u];
	}
	for (uint32_t r = nb * 4u * B; r < stripes; r++)
		acc = xxh_round_pre(acc, reinterpret_cast<const uint32_t *>(P + 64u * (r >> 2))[r & 3u]);
	const uint32_t a1 = __shfl_down(acc, 1, 4), a2 = __shfl_down(acc, 2, 4), a3 = __shfl_down(acc, 3, 4);
	if (q != 0 || !valid)
		return;
	const uint32_t frame = frame_list ? frame_list[lf] : lf;
	const uint8_t *f = src + (uint64_t)frame * stride;
	uint32_t h = stripes ? rotl32(acc, 1) + rotl32(a1, 7) + rotl32(a2, 12) + rotl32(a3, 18) : seed + XP5;
	h += len;
	uint32_t i = 8u * stripes;
	const uint32_t rem_bytes = len - 16u * stripes;
	uint32_t bb = 0;
	for (; bb + 4u <= rem_bytes; bb += 4u, i += 2u)
		h = rotl32(h + be_pair(sample_at<W>(f, i), sample_at<W>(f, i + 1u)) * XP3, 17) * XP4;
	if (bb < rem_bytes) {
		const uint32_t s0 = sample_at<W>(f, i);
		h = rotl32(h + ((s0 >> 8) & 0xFFu) * XP5, 11) * XP1;
		h = rotl32(h + (s0 & 0xFFu) * XP5, 11) * XP1;
	}
	h ^= h >> 15;
	h *= XP2;
	h ^= h >> 13;
	h *= XP3;
	h ^= h >> 16;
	out[frame] = h;
}


// ---------------------------------------------------------------------
// Per-frame Rice parameter selection (build-defined rule; oracle
// orc_select_rice_k): total_k = n(k+1) + sum_i min(v_i >> k, 16), v = m + 1.
// The 129-bin histogram of enc_common.h (auto_term) is a sufficient statistic.
// ---------------------------------------------------------------------
// Frames above AUTO_MAX_SPF segments (the fused path's limit), passes that
// store a model, and IWT passes (over their coefficients): a frame takes one
// workgroup per RICE_SLICE samples (a 4 Mi-sample frame 64), which read its
// 4096-sample chunks interleaved.  Each workgroup builds its histogram in LDS
// with the fused path's layout (enc_kernel.h AUTO: the 129 bins of
// enc_common.h auto_term, one 32-bit counter per bin and lane, so a wave's
// atomics never share a bank) and adds the non-zero bins to the frame's
// global histogram; the workgroup that arrives last (a per-frame counter)
// takes the argmin of the 16 totals, ties to the smaller k, and writes g.
// (4, 8 or 32 chunks per workgroup instead of 16 measured the same.)
#define RICE_SLICE (256u * AIRS_PT * 16u)
#define RICE_HSTRIDE 132u // global words per launch frame: 129 bins, the arrival counter, pad
template <int W, int PRE>
__global__ __launch_bounds__(256) void select_rice_hist_kernel(const uint8_t *src, uint64_t stride, uint32_t div,
								const uint64_t *ptrs, uint32_t n, const uint32_t *flist,
								uint32_t fadd, uint32_t fmul, uint32_t *ghist, uint32_t *out_g)
{
	__shared__ uint32_t H[AUTO_BINS * 64u];
	__shared__ uint32_t s_bin[AUTO_BINS];
	__shared__ uint32_t s_tot[16][17];
	__shared__ uint32_t s_last;
	const uint32_t tid = threadIdx.x, lane = tid & 63u;
	const uint32_t frame = flist ? flist[blockIdx.x] : fadd + blockIdx.x * fmul;
	if (frame == AIRS_NO_FRAME)
		return;
	// the frame's samples, or (IWT passes) its coefficients in the work buffer
	// of the launch's model addressing: ptrs[j], or src + (frame / div) * stride
	const uint8_t *f = ptrs ? reinterpret_cast<const uint8_t *>(ptrs[blockIdx.x]) : src + (uint64_t)(frame / div) * stride;
	for (uint32_t i = tid; i < sizeof(H) / 16u; i += 256u)
		reinterpret_cast<uint4 *>(H)[i] = make_uint4(0u, 0u, 0u, 0u);
	// lane's counter of bin b at byte hbase + 256 (b + 1016): b from the float bits
	const uint32_t hbase = (uint32_t)(uintptr_t)H + 4u * lane - 1016u * 256u;
	__syncthreads();
	// one 16-sample group per lane and step (the step count is uniform: the
	// shuffle below needs every lane of the wave).  Workgroup y takes the
	// frame's 4096-sample chunks y, y + G, y + 2G, ... (G = gridDim.y), so at
	// any time the frame's workgroups read one contiguous span
	const uint32_t G = gridDim.y;
	constexpr uint32_t CHN = 256u * AIRS_PT; // samples per chunk
	const uint32_t chunks = (n + CHN - 1u) / CHN, y = blockIdx.y;
	const uint32_t steps = chunks > y ? (chunks - y + G - 1u) / G : 0u;
	const uint32_t step_n = G * CHN; // samples between this workgroup's chunks
	auto bin1 = [&](uint32_t u, uint32_t inc) {
		const int32_t d = (int32_t)(u << 16) >> 16;
		const uint32_t v = (uint32_t)((d << 1) ^ (d >> 31)) + 1u;
		const uint32_t ha = ((__float_as_uint((float)v) >> 20) << 8) + hbase;
		__hip_atomic_fetch_add(reinterpret_cast<lds_u32 *>((uintptr_t)ha), inc, __ATOMIC_RELAXED,
				       __HIP_MEMORY_SCOPE_WORKGROUP);
	};
	if (((uintptr_t)f & 15u) == 0u && n % CHN == 0u) {
		// whole aligned chunks: straight-line loads of the raw words, every
		// lane also loading the sample before its group (lane 0 uses it)
		constexpr uint32_t RW = W; // uint4 per lane: 16 samples of W bytes
		uint4 ra[RW], rb[RW];
		uint32_t pa, pb;
		auto ldraw = [&](uint4 (&r)[RW], uint32_t &p0, uint32_t b) {
			const uint4 *q = reinterpret_cast<const uint4 *>(f + (size_t)b * W);
#pragma unroll
			for (uint32_t i = 0; i < RW; i++)
				r[i] = q[i];
			p0 = PRE == PRE_DIFF ? sample_at<W>(f, b ? b - 1u : 0u) : 0u;
		};
		auto binraw = [&](const uint4 (&r)[RW], uint32_t p0, uint32_t inc) {
			uint32_t x[AIRS_PT];
#pragma unroll
			for (uint32_t i = 0; i < RW; i++) {
				const uint32_t w[4] = {r[i].x, r[i].y, r[i].z, r[i].w};
#pragma unroll
				for (uint32_t e = 0; e < 4u; e++) {
					if (W == 2) {
						x[8u * i + 2u * e] = w[e] & 0xFFFFu;
						x[8u * i + 2u * e + 1u] = w[e] >> 16;
					} else {
						x[4u * i + e] = w[e] & 0xFFFFu;
					}
				}
			}
			uint32_t prev = 0u;
			if (PRE == PRE_DIFF) {
				// the sample before this lane's group: the previous lane's last one
				prev = __shfl_up(x[AIRS_PT - 1], 1, 64);
				if (lane == 0u)
					prev = p0;
			}
#pragma unroll
			for (int j = 0; j < AIRS_PT; j++)
				bin1(PRE == PRE_DIFF ? x[j] - (j ? x[j - 1] : prev) : x[j], inc);
		};
		// two chunks per iteration, both loaded before either is binned, in
		// one basic block so that the waits count exactly (a prefetch carried
		// across iterations, or the second chunk binned under a branch, ended
		// in over-waits); an odd last step bins its chunk twice, the second
		// time adding 0
		uint32_t base = y * CHN + tid * AIRS_PT;
		for (uint32_t st = 0; st < steps; st += 2u, base += 2u * step_n) {
			const bool two = st + 1u < steps;
			ldraw(ra, pa, base);
			ldraw(rb, pb, two ? base + step_n : base);
			binraw(ra, pa, 1u);
			binraw(rb, pb, two ? 1u : 0u);
		}
	} else {
		// any other frame: 16 samples per lane and step, guarded
		for (uint32_t st = 0, base = y * CHN + tid * AIRS_PT; st < steps; st++, base += step_n) {
			uint32_t x[AIRS_PT];
			load16<W>(f, base, n, x);
			uint32_t prev = 0u;
			if (PRE == PRE_DIFF) {
				prev = __shfl_up(x[AIRS_PT - 1], 1, 64);
				if (lane == 0u)
					prev = base > 0u && base - 1u < n ? sample_at<W>(f, base - 1u) : 0u;
			}
#pragma unroll
			for (int j = 0; j < AIRS_PT; j++)
				if (base + j < n)
					bin1(PRE == PRE_DIFF ? x[j] - (j ? x[j - 1] : prev) : x[j], 1u);
		}
	}
	__syncthreads();
	// bin totals: threads 2r, 2r+1 sum the halves of row r < 128; wave 0 row 128
	{
		const uint32_t r = tid >> 1, h = tid & 1u;
		const uint4 *row = reinterpret_cast<const uint4 *>(H + r * 64u + h * 32u);
		uint32_t t = 0u;
#pragma unroll
		for (uint32_t q = 0; q < 8u; q++) {
			const uint4 v = row[(q + r) & 7u];
			t += v.x + v.y + v.z + v.w;
		}
		t += __shfl_xor(t, 1, 64);
		if (h == 0u)
			s_bin[r] = t;
		if (tid < 64u) {
			uint32_t t128 = H[128u * 64u + lane];
#pragma unroll
			for (uint32_t o = 32u; o; o >>= 1)
				t128 += __shfl_xor(t128, (int)o, 64);
			if (lane == 0u)
				s_bin[128] = t128;
		}
	}
	__syncthreads();
	// The frame's histogram and arrival counter live in device memory and are
	// touched by agent-scope atomics only, which execute at the memory side
	// (MI355X_MICROARCH.md: atomics drop the line from the XCD's L2): no
	// fence (__threadfence writes back and invalidates the caches, ~14 us per
	// workgroup at four per CU).  Each bin add returns before the barrier, the
	// arrival add after it; the last arrival reads the bins by exchanges, also
	// at the memory side (an add of 0 may be turned into a cached load).
	// This ordering is the hardware's, not the memory model's: relaxed
	// atomics promise none.  It holds on gfx950 (returning agent-scope
	// atomics are performed at the memory side in the order the wave waits
	// for them); any other target must add release/acquire here first
	// (ADVICE r5), hence the guard below.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "select_rice_hist_kernel's fence-free hand-off is verified for gfx950 only"
#endif
	uint32_t *gh = ghist + (uint64_t)blockIdx.x * RICE_HSTRIDE;
	if (tid < AUTO_BINS && s_bin[tid]) {
		const uint32_t r = __hip_atomic_fetch_add(&gh[tid], s_bin[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		asm volatile("" ::"v"(r)); // a returning add: it has been performed once the value is back
	}
	__syncthreads();
	if (tid == 0u)
		s_last = __hip_atomic_fetch_add(&gh[AUTO_BINS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
			 gridDim.y - 1u;
	__syncthreads();
	if (!s_last)
		return;
	// the last slice: the frame's 16 candidate totals n(k+1) + sum_b h_b term(b, k)
	if (tid < AUTO_BINS)
		s_bin[tid] = __hip_atomic_exchange(&gh[tid], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	__syncthreads();
	{
		const uint32_t k = tid & 15u, sl = tid >> 4;
		uint32_t part = 0u; // <= 16 n < 2^28
		for (uint32_t b = sl; b < AUTO_BINS; b += 16u)
			part += s_bin[b] * auto_term(b, k);
		s_tot[k][sl] = part;
	}
	__syncthreads();
	if (tid < 16u) {
		uint32_t t = n * (tid + 1u);
#pragma unroll
		for (uint32_t sl = 0; sl < 16u; sl++)
			t += s_tot[tid][sl];
		s_tot[tid][16] = t;
	}
	__syncthreads();
	if (tid == 0u) {
		uint32_t best = 0u;
		for (uint32_t k = 1u; k < 16u; k++)
			if (s_tot[k][16] < s_tot[best][16])
				best = k;
		out_g[frame] = 1u << best;
	}
}

// ---------------------------------------------------------------------
// Batch fallback path on the device (cmp_gpu_compress, contexts with the
// uncompressed fallback or frames that can fail): the context state machine
// of compress_engine / cmp_compress_generic (reference cmp.c:228-246,
// 342-393) runs here, one thread per context, so that a batch needs no host
// round trip per acquisition step.  Per step a: fb_step_kernel resolves step
// a-1 (outcome -> sequence number, fallback decision, identifier draws) and
// plans step a (primary or secondary pass -> the launch lists of the two
// encode launches); fb_copy_kernel writes the raw NONE + UNCOMPRESSED frames
// of step a-1's fallbacks (and their model store).
// ---------------------------------------------------------------------
__global__ void fb_step_kernel(airs_fb_step a)
{
	const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
	if (c >= a.num_ctx)
		return;
	uint32_t seq = a.state[2u * c], msize = a.state[2u * c + 1u];
	if (a.prev >= 0) {
		const uint32_t f = c * a.fpc + (uint32_t)a.prev;
		uint8_t fb = 0;
		if (a.kind[f]) {
			const uint32_t v = a.status[f];
			if (v <= a.err_floor) {
				seq++; // compress_engine succeeded (cmp.c:336)
			} else if (a.fb_eligible && v == a.err_small) {
				// cmp.c:375-392: reset (a draw), then the frame again as a
				// primary NONE + UNCOMPRESSED pass (its own reset: a draw)
				fb = 1;
				a.draws[f] = (uint8_t)(a.draws[f] + 2u);
				msize = a.packed;
				if (a.raw_size > 0xFFFFFFu) {
					a.status[f] = a.err_too_large; // header.c: size field
					seq = 0;
				} else {
					a.status[f] = a.raw_size;
					seq = 1;
				}
			}
			// any other error: the sequence number stays (cmp.c returns early)
		}
		a.fb[f] = fb;
	}
	if (a.cur >= 0) {
		const uint32_t f = c * a.fpc + (uint32_t)a.cur;
		uint32_t lp = AIRS_NO_FRAME, ls = AIRS_NO_FRAME;
		uint8_t kind = 0, draws = 0;
		if (seq == 0 || seq > a.iters) { // cmp.c:228-237: reset, primary pass
			seq = 0;
			msize = a.packed;
			draws = 1;
			kind = 1;
			lp = f;
		} else if (a.model_needed && msize != a.packed) { // cmp.c:244-245
			a.status[f] = a.err_mismatch;
		} else {
			kind = 2;
			ls = f;
		}
		a.flist_p[c] = lp;
		a.flist_s[c] = ls;
		a.seqs[f] = (uint8_t)seq;
		a.kind[f] = kind;
		a.draws[f] = draws;
	}
	a.state[2u * c] = seq;
	a.state[2u * c + 1u] = msize;
}

// raw frames of step `prev`'s fallbacks: header (16 B), the samples as
// big-endian 16-bit words, the checksum; the model takes the samples (the
// fallback is a primary pass: cmp.c:304-306).  Block (c, j) covers samples
// [j * 2048, (j + 1) * 2048) of context c's frame.
template <int W>
__global__ __launch_bounds__(256) void fb_copy_kernel(airs_fb_step a)
{
	const uint32_t c = blockIdx.x, f = c * a.fpc + (uint32_t)a.prev;
	if (!a.fb[f])
		return;
	const uint32_t n = a.n, i0 = blockIdx.y * 2048u + threadIdx.x * 8u;
	const uint8_t *fs = (const uint8_t *)a.src + (uint64_t)f * a.src_stride;
	uint8_t *fd = (uint8_t *)a.dst + (uint64_t)f * a.dst_stride;
	uint16_t *fm = nullptr;
	if (a.model_needed)
		fm = (uint16_t *)(a.model_ptrs ? (uint8_t *)(uintptr_t)a.model_ptrs[c]
					       : (uint8_t *)a.model + (uint64_t)c * a.model_stride);
	uint32_t x[8];
#pragma unroll
	for (uint32_t q = 0; q < 8u; q++) {
		const uint32_t i = i0 + q;
		x[q] = i < n ? (W == 2 ? (uint32_t)reinterpret_cast<const uint16_t *>(fs)[i]
				       : reinterpret_cast<const uint32_t *>(fs)[i] & 0xFFFFu)
			     : 0u;
	}
	if (i0 + 8u <= n) { // 16 bytes at 16 + 2 i0: 16-byte aligned (dst is 8-byte, i0 a multiple of 8)
		uint4 o;
		o.x = __builtin_bswap32(x[0] << 16 | x[1]);
		o.y = __builtin_bswap32(x[2] << 16 | x[3]);
		o.z = __builtin_bswap32(x[4] << 16 | x[5]);
		o.w = __builtin_bswap32(x[6] << 16 | x[7]);
		uint8_t *p = fd + 16u + 2u * i0;
		if (((uintptr_t)p & 15u) == 0u) {
			*reinterpret_cast<uint4 *>(p) = o;
		} else {
			reinterpret_cast<uint2 *>(p)[0] = make_uint2(o.x, o.y);
			reinterpret_cast<uint2 *>(p)[1] = make_uint2(o.z, o.w);
		}
	} else {
		for (uint32_t q = 0; q < 8u && i0 + q < n; q++) {
			fd[16u + 2u * (i0 + q)] = (uint8_t)(x[q] >> 8);
			fd[17u + 2u * (i0 + q)] = (uint8_t)x[q];
		}
	}
	if (fm) {
		for (uint32_t q = 0; q < 8u && i0 + q < n; q++)
			fm[i0 + q] = (uint16_t)x[q];
	}
	if (blockIdx.y == 0 && threadIdx.x == 0) {
		uint32_t h[5];
		header_words(h, a.raw_size, 2u * n, 0u, 0u, PRE_NONE, a.checksum ? 1u : 0u, ENC_RAW, 0u, 0u, 0u);
#pragma unroll
		for (uint32_t w = 0; w < 4u; w++)
			reinterpret_cast<uint32_t *>(fd)[w] = __builtin_bswap32(h[w]);
		if (a.checksum) {
			const uint32_t ck = a.checksums[f];
			for (uint32_t b = 0; b < 4u; b++)
				fd[16u + 2u * n + b] = (uint8_t)(ck >> (24u - 8u * b));
		}
	}
}

// ---------------------------------------------------------------------
// Frame packing for the multi-GPU gather (cmp_gpu_pack_frames, shard.py):
// the frames of a strided batch buffer, back to back at 8-byte aligned
// offsets, reading only the compressed bytes (rounded up to 8).
// ---------------------------------------------------------------------
__global__ __launch_bounds__(1024) void pack_scan_kernel(const uint32_t *sizes, uint32_t num, uint32_t err_floor,
							 uint64_t *offsets)
{
	__shared__ uint64_t s_w[16];
	__shared__ uint64_t s_carry;
	const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
	if (t == 0)
		s_carry = 0;
	__syncthreads();
	for (uint32_t base = 0; base < num; base += 1024u) {
		const uint32_t i = base + t;
		const uint32_t sz = i < num ? sizes[i] : 0u;
		const uint64_t v = (sz > err_floor) ? 0u : ((uint64_t)sz + 7u) & ~7ull;
		uint64_t inc = v;
#pragma unroll
		for (uint32_t d = 1; d < 64u; d <<= 1) {
			const uint64_t o = __shfl_up(inc, d, 64);
			inc += lane >= d ? o : 0u;
		}
		if (lane == 63u)
			s_w[w] = inc;
		__syncthreads();
		uint64_t pre = s_carry;
		for (uint32_t k = 0; k < w; k++)
			pre += s_w[k];
		if (i < num)
			offsets[i] = pre + inc - v;
		__syncthreads();
		if (t == 1023u)
			s_carry = pre + inc;
		__syncthreads();
	}
	if (t == 0)
		offsets[num] = s_carry;
}

__global__ __launch_bounds__(256) void pack_copy_kernel(const uint8_t *src, uint64_t stride, const uint32_t *sizes,
							uint32_t err_floor, const uint64_t *offsets, uint8_t *out)
{
	const uint32_t f = blockIdx.x, sz = sizes[f];
	if (sz > err_floor)
		return;
	const uint32_t nw = (sz + 7u) >> 3; // 8-byte words of the frame
	const uint2 *s8 = reinterpret_cast<const uint2 *>(src + (uint64_t)f * stride);
	uint2 *o8 = reinterpret_cast<uint2 *>(out + offsets[f]);
	// blocks of 1024 words, grid-stride over y (gridDim.y is capped at 65535)
	for (uint32_t b = blockIdx.y; (uint64_t)b * 1024u < nw; b += gridDim.y)
		for (uint32_t j = b * 1024u + threadIdx.x; j < nw && j < (b + 1u) * 1024u; j += 256u)
			o8[j] = s8[j];
}

// identifier patch after fallback resolution (header bytes 8..13)
__global__ void patch_ids_kernel(uint8_t *dst, uint64_t stride, uint32_t num, uint32_t fadd, uint32_t fmul,
				 const uint64_t *ids, const uint32_t *status)
{
	const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
	if (j >= num)
		return;
	const uint32_t f = fadd + j * fmul;
	if (status && status[f] > ERRV(128u))
		return;
	uint8_t *p = dst + (uint64_t)f * stride + 8u;
	const uint64_t id = ids[j];
	for (int b = 0; b < 6; b++)
		p[b] = (uint8_t)(id >> (40 - 8 * b));
}

// The speculative walk's commit (airs_dev_commit_*), one workgroup: flags[c]
// = 1 when a frame of context c (frames c*fpc ..) has an error status, the
// fault count, then (after a system-scope fence) the signal `seq`.  Then it
// waits for the host's release (bounded: `ticks` of the 100 MHz clock, ~1 s)
// and, if the release says so, writes the identifiers the host put in the
// block into the headers of the frames without an error (as
// patch_ids_kernel).  Last, its acknowledgement: whether it patched, so that
// a host whose release came after the kernel gave up patches the headers
// itself.  The stream's next work waits behind it, and no host
// launch is needed.
__global__ void commit_kernel(const uint32_t *status, uint32_t num_ctx, uint32_t fpc, const uint32_t *ticket,
			      volatile uint32_t *hco, uint32_t seq, uint8_t *dst, uint64_t dst_stride, uint64_t ticks)
{
	__shared__ uint32_t s_mode;
	volatile uint8_t *flags = reinterpret_cast<volatile uint8_t *>(hco) + AIRS_HCO_FLAGS;
	for (uint32_t c = threadIdx.x; c < num_ctx; c += blockDim.x) {
		uint32_t any = 0u;
		for (uint32_t a = 0; a < fpc; a++)
			any |= status[(uint64_t)c * fpc + a] > ERRV(128u) ? 1u : 0u;
		flags[c] = (uint8_t)any;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		hco[AIRS_HCO_FAULT] = ticket[AIRS_FAULT_WORD];
		__threadfence_system();
		hco[AIRS_HCO_SEQ] = seq;
		const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
		uint32_t mode = 0u;
		for (;;) {
			if (__hip_atomic_load(hco + AIRS_HCO_GO, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == seq) {
				mode = hco[AIRS_HCO_MODE];
				break;
			}
			if (__builtin_amdgcn_s_memrealtime() - t0 > ticks)
				break; // no release: leave the headers alone
			__builtin_amdgcn_s_sleep(8);
		}
		s_mode = mode;
	}
	__syncthreads();
	if (s_mode != 1u) {
		if (threadIdx.x == 0) {
			__threadfence_system();
			hco[AIRS_HCO_ACK] = (seq & 0x7FFFFFFFu) << 1;
		}
		return;
	}
	const volatile uint64_t *ids =
		reinterpret_cast<const volatile uint64_t *>(reinterpret_cast<volatile uint8_t *>(hco) + AIRS_HCO_IDS);
	const uint32_t total = num_ctx * fpc;
	for (uint32_t f = threadIdx.x; f < total; f += blockDim.x) {
		if (status[f] > ERRV(128u))
			continue;
		uint8_t *p = dst + (uint64_t)f * dst_stride + 8u;
		const uint64_t id = ids[f];
		for (int b = 0; b < 6; b++)
			p[b] = (uint8_t)(id >> (40 - 8 * b));
	}
	__syncthreads(); // every header written (the fence below covers the block's stores)
	if (threadIdx.x == 0) {
		__threadfence_system();
		hco[AIRS_HCO_ACK] = ((seq & 0x7FFFFFFFu) << 1) | 1u;
	}
}

// ---------------------------------------------------------------------
// counter-hash synthetic frames (oracle orc_synth_u16 / orc_synth_i32)
// ---------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t z)
{
	z += 0x9E3779B97F4A7C15ull;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

template <int W>
__global__ void synth_kernel(uint8_t *dst, uint64_t seed, uint32_t frame0, uint32_t n, uint64_t stride,
			     uint32_t W_noise)
{
	const uint32_t frame = blockIdx.y;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		const uint64_t h = splitmix64(seed ^ ((uint64_t)(frame0 + frame) << 32) ^ i);
		const uint32_t t = i & 0xFFFFu;
		const int32_t tri = (int32_t)((t < 32768u ? t : 65536u - t) >> 3);
		uint32_t v;
		if (((h >> 20) & 1023u) == 0u) {
			v = (uint32_t)((h >> 32) & 0xFFFFu);
		} else {
			int32_t xv = 16384 + tri + (int32_t)((h & 0xFFFFu) % (2u * W_noise + 1u)) - (int32_t)W_noise;
			v = (uint32_t)min(max(xv, 0), 65535);
		}
		uint8_t *f = dst + (uint64_t)frame * stride;
		if (W == 2)
			reinterpret_cast<uint16_t *>(f)[i] = (uint16_t)v;
		else
			reinterpret_cast<uint32_t *>(f)[i] = ((uint32_t)(h >> 48) << 16) | v;
	}
}

} // namespace airs

// =====================================================================
// device layer (C ABI, see airs_dev.h)
// =====================================================================
using namespace airs;

static thread_local char g_err[256];

#if AIRS_ABLATE
// Ablation builds only (scripts/build_exp.sh -DAIRS_ABLATE=1): the AIRS_DBG
// switches of enc_common.h DBG(), set by the benchmark harness
// (scripts/kbench.py) through this entry point; the product build has none.
static uint32_t g_dbg;
static char g_dbgts_path[512];
// AIRS_DBGTS_RING=R: the timeline keeps the last R launches (slot = launch
// number mod R, one block of 8 stamps per segment each), zeroed once at
// allocation so that back-to-back launches see no extra memset
static uint32_t g_dbgts_ring = 1u, g_dbgts_launch;
extern "C" void airs_dev_set_debug(uint32_t bits, const char *timeline_path)
{
	g_dbg = bits;
	snprintf(g_dbgts_path, sizeof(g_dbgts_path), "%s", timeline_path ? timeline_path : "");
	const char *r = getenv("AIRS_DBGTS_RING");
	g_dbgts_ring = r && atoi(r) > 0 ? (uint32_t)atoi(r) : 1u;
	g_dbgts_launch = 0u;
}
#endif

static uint32_t hip_fail(hipError_t e, const char *what)
{
	snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
	fprintf(stderr, "airscmp: %s\n", g_err);
	return ERRV(E_GENERIC);
}

#define HIPCHECK(x)                                 \
	do {                                        \
		hipError_t _e = (x);                \
		if (_e != hipSuccess)               \
			return hip_fail(_e, #x);    \
	} while (0)

struct airs_dev_engine {
	hipStream_t stream;
	uint64_t *agg;
	uint64_t *tail;
	size_t gran_cap; // segments
	uint32_t *ticket;
	uint32_t ticket_base;
	uint32_t walk_ticket_base; // ticket[AIRS_WALK_TICKET] before the next segment walk
	uint32_t epoch;
	void *scratch[AIRS_NSLOT];
	size_t scratch_cap[AIRS_NSLOT];
	uint64_t *dbgts; // debug timeline (AIRS_DBG bit 65536)
	size_t dbgts_n;
	uint64_t *ktot; // fused Rice selection: 16 candidate granules per segment
	size_t ktot_cap;
	uint32_t *rhist; // sliced Rice selection: 128 bins per frame
	size_t rhist_cap; // frames
	void *pinned; // page-locked host scratch (read-backs, identifier uploads)
	size_t pinned_cap;
	volatile uint32_t *hco; // coherent page-locked block (AIRS_HCO_*), written in-stream
	uint32_t hco_seq;       // the last sequence word asked for
	uint32_t hco_released;  // the last sequence word released (airs_dev_commit_release)
	uint64_t commit_ticks;  // the commit kernel's wait for the release (100 MHz ticks)
	uint64_t commit_polls;  // the host's wait for the commit kernel's signal (pause loops)
	// a release with identifiers whose patch is not yet confirmed by the
	// kernel's acknowledgement (checked at the next stream wait): its seq (0:
	// none), the frames and the identifiers (page-locked: patch_ids_kernel
	// reads them over the bus if the kernel gave up)
	uint32_t commit_total;   // the frames of the commit kernel last begun
	void *commit_dst;
	uint64_t commit_dst_stride;
	const uint32_t *commit_status;
	uint32_t pend_seq, pend_total, pend_buf; // the pending release (pend_seq 0: none)
	void *pend_dst;
	uint64_t pend_dst_stride;
	const uint32_t *pend_status;
	uint64_t *commit_ids[2]; // two buffers: a patch queued for release N reads its own
	size_t commit_ids_cap[2];
	// cmp_gpu_engine_set_option (include/cmp_gpu.h)
	uint32_t opt_exclusive;     // CMP_GPU_OPT_EXCLUSIVE
	uint32_t opt_walk_segment;  // CMP_GPU_OPT_WALK_SEGMENT: 0, 2048 or 4096
	uint32_t opt_no_ctx_walk;   // CMP_GPU_OPT_NO_CONTEXT_WALK
};

extern "C" uint32_t airs_dev_set_option(struct airs_dev_engine *e, uint32_t option, uint32_t value)
{
	if (!e)
		return ERRV(E_GENERIC);
	switch (option) {
	case AIRS_OPT_EXCLUSIVE:
		e->opt_exclusive = value ? 1u : 0u;
		return 0;
	case AIRS_OPT_WALK_SEGMENT:
		if (value != 0u && value != 2048u && value != 4096u)
			return ERRV(E_PARAMS_INVALID);
		e->opt_walk_segment = value;
		return 0;
	case AIRS_OPT_NO_CONTEXT_WALK:
		e->opt_no_ctx_walk = value ? 1u : 0u;
		return 0;
	default:
		return ERRV(E_PARAMS_INVALID);
	}
}

extern "C" int airs_dev_available(void)
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess)
		return 0;
	return n > 0;
}

extern "C" const char *airs_dev_last_error(void)
{
	return g_err;
}

static int commit_verify(struct airs_dev_engine *e);

extern "C" struct airs_dev_engine *airs_dev_engine_create(void *stream)
{
	if (!airs_dev_available()) {
		snprintf(g_err, sizeof(g_err), "no HIP device available");
		return nullptr;
	}
	airs_dev_engine *e = (airs_dev_engine *)calloc(1, sizeof(airs_dev_engine));
	if (!e)
		return nullptr;
	e->stream = (hipStream_t)stream;
	// 256 bytes of tickets and fault words, then the gather's status words
	const size_t tbytes = 256u + 16u * (AIRS_COLL_MAX_RANKS + 1u);
	if (hipMalloc(&e->ticket, tbytes) != hipSuccess || hipMemset(e->ticket, 0, tbytes) != hipSuccess) {
		free(e);
		return nullptr;
	}
	void *hf = nullptr;
	if (hipHostMalloc(&hf, AIRS_HCO_BYTES, hipHostMallocCoherent) != hipSuccess) {
		(void)hipFree(e->ticket);
		free(e);
		return nullptr;
	}
	e->hco = (volatile uint32_t *)hf;
	// the commit handshake's bounds; AIRS_TEST_COMMIT_TICKS / _POLLS shorten
	// them to force its give-up paths (tests only)
	e->commit_ticks = 100000000ull;
	e->commit_polls = 1ull << 26;
	if (const char *t = getenv("AIRS_TEST_COMMIT_TICKS"))
		e->commit_ticks = strtoull(t, nullptr, 10);
	if (const char *t = getenv("AIRS_TEST_COMMIT_POLLS"))
		e->commit_polls = strtoull(t, nullptr, 10);
	e->hco[AIRS_HCO_FAULT] = 0u;
	e->hco[AIRS_HCO_ACK] = 0u;
	e->hco[AIRS_HCO_SEQ] = 0u;
	e->hco[AIRS_HCO_GO] = 0u;
	e->epoch = 0;
	return e;
}

extern "C" void airs_dev_engine_destroy(struct airs_dev_engine *e)
{
	if (!e)
		return;
	(void)hipStreamSynchronize(e->stream);
	if (commit_verify(e))
		(void)hipStreamSynchronize(e->stream);
	(void)hipFree(e->agg);
	(void)hipFree(e->tail);
	(void)hipFree(e->ticket);
	(void)hipFree(e->dbgts);
	(void)hipFree(e->ktot);
	(void)hipFree(e->rhist);
	for (int i = 0; i < AIRS_NSLOT; i++)
		(void)hipFree(e->scratch[i]);
	if (e->pinned)
		(void)hipHostFree(e->pinned);
	for (int b = 0; b < 2; b++)
		if (e->commit_ids[b])
			(void)hipHostFree(e->commit_ids[b]);
	if (e->hco)
		(void)hipHostFree((void *)e->hco);
	free(e);
}

extern "C" void *airs_dev_host_scratch(struct airs_dev_engine *e, size_t bytes)
{
	if (e->pinned_cap < bytes) {
		(void)hipStreamSynchronize(e->stream); // a copy from or to the old buffer may be in flight
		if (e->pinned)
			(void)hipHostFree(e->pinned);
		e->pinned = nullptr;
		e->pinned_cap = 0;
		const size_t want = bytes < 65536 ? 65536 : bytes + bytes / 4;
		const hipError_t he = hipHostMalloc(&e->pinned, want, hipHostMallocDefault);
		if (he != hipSuccess) {
			(void)hip_fail(he, "hipHostMalloc (engine host scratch)");
			return nullptr;
		}
		e->pinned_cap = want;
	}
	return e->pinned;
}

extern "C" void *airs_dev_engine_stream(struct airs_dev_engine *e)
{
	return e ? (void *)e->stream : nullptr;
}

extern "C" uint64_t *airs_dev_coll(struct airs_dev_engine *e)
{
	return e ? reinterpret_cast<uint64_t *>(e->ticket + 64) : nullptr;
}

extern "C" void *airs_dev_scratch(struct airs_dev_engine *e, int slot, size_t bytes)
{
	if (slot < 0 || slot >= AIRS_NSLOT)
		return nullptr;
	if (e->scratch_cap[slot] < bytes) {
		(void)hipStreamSynchronize(e->stream);
		(void)hipFree(e->scratch[slot]);
		e->scratch[slot] = nullptr;
		e->scratch_cap[slot] = 0;
		size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
		const hipError_t he = hipMalloc(&e->scratch[slot], want);
		if (he != hipSuccess) {
			(void)hip_fail(he, "hipMalloc (engine scratch)");
			return nullptr;
		}
		e->scratch_cap[slot] = want;
	}
	return e->scratch[slot];
}

// Words of one LDS chunk image: the longest codeword (bits per sample) the
// pass can emit: UNCOMPRESSED 16; ZERO k+17 (escape, and the longest
// non-escape code) with k = floor(log2 g), 32 when g varies per frame
// (g = 0 here); MULTI up to 48 (two pieces)
static uint32_t image_words(uint32_t encoder_type, uint32_t g)
{
	uint32_t maxbits = 48u;
	if (encoder_type == ENC_RAW) {
		maxbits = 16u;
	} else if (encoder_type == ENC_ZERO) {
		uint32_t kk = 15u;
		if (g) {
			kk = 0u;
			while ((2u << kk) <= g && kk < 31u)
				kk++;
		}
		maxbits = kk + 17u < 32u ? kk + 17u : 32u;
	}
#ifdef AIRS_IMG_BITS // experiments only: images too small for the worst case
	maxbits = AIRS_IMG_BITS;
#endif
	const uint32_t words = AIRS_SEG * maxbits / 32u + 4u;
	return (words + 3u) & ~3u;
}

// Rice ZERO or MULTI (g a power of two): the passes the walks code
static bool walk_rice(uint32_t enc, uint32_t g)
{
	return (enc == ENC_ZERO || enc == ENC_MULTI) && g && (g & (g - 1u)) == 0u;
}

// Longest codeword (bits) a Rice pass emits with these parameters (the
// outlier clamped as make_coder does); sizes the context walk's images
static uint32_t code_max_bits(uint32_t enc, uint32_t g, uint32_t outlier_param)
{
	if (enc == ENC_RAW || !g)
		return enc == ENC_RAW ? 16u : 48u;
	uint32_t k = 0u;
	while ((2u << k) <= g && k < 31u)
		k++;
	if (enc == ENC_ZERO)
		return k + 17u;
	uint64_t limit = (uint64_t)g + (uint64_t)(31u - k) * g;
	limit = limit > 8u ? limit - 8u : 0u;
	const uint64_t outl = outlier_param < limit ? outlier_param : limit;
	const uint64_t nonesc = outl ? ((outl - 1u) >> k) + k + 1u : 0u;
	const uint64_t esc = outl <= 65535u ? ((outl + 7u) >> k) + k + 1u + 16u : 0u;
	const uint64_t mb = nonesc > esc ? nonesc : esc;
	return mb < 48u ? (uint32_t)mb : 48u;
}

// launch epoch tag of the look-back granules (never 0: zeroed granules never match)
static uint32_t next_epoch(airs_dev_engine *e)
{
	e->epoch = (e->epoch + 1u) & 0x7FFFFFFFu;
	if (e->epoch == 0)
		e->epoch = 1;
	return e->epoch;
}

static uint32_t ensure_granules(airs_dev_engine *e, size_t segs)
{
	if (segs <= e->gran_cap)
		return 0;
	HIPCHECK(hipStreamSynchronize(e->stream));
	(void)hipFree(e->agg);
	(void)hipFree(e->tail);
	e->agg = e->tail = nullptr;
	size_t want = segs + segs / 2 + 1024;
	HIPCHECK(hipMalloc(&e->agg, want * sizeof(uint64_t)));
	HIPCHECK(hipMalloc(&e->tail, want * sizeof(uint64_t)));
	// epoch tags start at 1, so zeroed granules never match
	HIPCHECK(hipMemset(e->agg, 0, want * sizeof(uint64_t)));
	HIPCHECK(hipMemset(e->tail, 0, want * sizeof(uint64_t)));
	e->gran_cap = want;
	return 0;
}

template <int W, int PRE, int ENC, bool RICE, int MODEL>
static void launch_encode(const KArgs &k, bool full, uint32_t grid, hipStream_t s)
{
	if constexpr (ENC == ENC_ZERO && RICE && MODEL == 0 && (PRE == PRE_NONE || PRE == PRE_DIFF)) {
		if (k.ktot) { // fused per-frame Rice selection (frame barrier: never persistent)
#ifndef AIRS_RICE_AUTO
#define AIRS_RICE_AUTO 1
#endif
			// the Rice kernel with the candidate barrier (enc_rice.hip)
			if (AIRS_RICE_AUTO && W == 2 && full && rice_auto_encode(k, PRE, s))
				return;
			size_t lds = (size_t)2u * (k.img_words + 4u) * 4u; // two images (enc_kernel.h NIMG)
			lds = lds > AUTO_BINS * 64u * 4u ? lds : AUTO_BINS * 64u * 4u; // the histogram
			if (full)
				launch_segments(encode_kernel<W, PRE, ENC, RICE, MODEL, true, true>, k, grid, lds, s);
			else
				launch_segments(encode_kernel<W, PRE, ENC, RICE, MODEL, false, true>, k, grid, lds, s);
			return;
		}
	}
#ifndef AIRS_RICE
#define AIRS_RICE 1
#endif
	// the Rice/ZERO frame kernel (enc_rice.hip)
	if constexpr (AIRS_RICE && W == 2 && (PRE == PRE_NONE || PRE == PRE_DIFF) && ENC == ENC_ZERO && RICE &&
		      MODEL == 0) {
		if (full && rice_encode(k, PRE, s, false))
			return;
	}
	const size_t lds = (size_t)seg_images(W, MODEL) * (k.img_words + 4u) * 4u;
#ifdef AIRS_EXP_ONLY
	// experiment builds: only the benchmark kernels (u16/i16, DIFF, ZERO, Rice, FULL)
	if constexpr (!(W == 2 && PRE == PRE_DIFF && ENC == ENC_ZERO && RICE && MODEL == 0)) {
		return;
	} else {
		if (full)
			launch_segments(encode_kernel<W, PRE, ENC, RICE, MODEL, true>, k, grid, lds, s);
		return;
	}
#else
	if (full)
		launch_segments(encode_kernel<W, PRE, ENC, RICE, MODEL, true>, k, grid, lds, s);
	else
		launch_segments(encode_kernel<W, PRE, ENC, RICE, MODEL, false>, k, grid, lds, s);
#endif
}

template <int W, int PRE, int MODEL>
static void dispatch_enc(const KArgs &k, uint32_t enc, bool rice, bool full, uint32_t grid, hipStream_t s)
{
	switch (enc) {
	case ENC_RAW:
		launch_encode<W, PRE, ENC_RAW, true, MODEL>(k, full, grid, s);
		break;
	case ENC_ZERO:
		if (rice)
			launch_encode<W, PRE, ENC_ZERO, true, MODEL>(k, full, grid, s);
		else
			launch_encode<W, PRE, ENC_ZERO, false, MODEL>(k, full, grid, s);
		break;
	default:
		if (rice)
			launch_encode<W, PRE, ENC_MULTI, true, MODEL>(k, full, grid, s);
		else
			launch_encode<W, PRE, ENC_MULTI, false, MODEL>(k, full, grid, s);
		break;
	}
}

template <int W>
static void dispatch_pre(const KArgs &k, uint32_t pre, uint32_t enc, bool rice, bool full, uint32_t model_mode,
			 uint32_t grid, hipStream_t s)
{
	if (pre == PRE_MODEL) {
		dispatch_enc<W, PRE_MODEL, AIRS_MODEL_UPDATE>(k, enc, rice, full, grid, s);
	} else if (pre == PRE_IWT) {
		if (model_mode == AIRS_MODEL_STORE)
			dispatch_enc<W, PRE_IWT, AIRS_MODEL_STORE>(k, enc, rice, full, grid, s);
		else
			dispatch_enc<W, PRE_IWT, AIRS_MODEL_NONE>(k, enc, rice, full, grid, s);
	} else if (pre == PRE_DIFF) {
		if (model_mode == AIRS_MODEL_STORE)
			dispatch_enc<W, PRE_DIFF, AIRS_MODEL_STORE>(k, enc, rice, full, grid, s);
		else
			dispatch_enc<W, PRE_DIFF, AIRS_MODEL_NONE>(k, enc, rice, full, grid, s);
	} else {
		if (model_mode == AIRS_MODEL_STORE)
			dispatch_enc<W, PRE_NONE, AIRS_MODEL_STORE>(k, enc, rice, full, grid, s);
		else
			dispatch_enc<W, PRE_NONE, AIRS_MODEL_NONE>(k, enc, rice, full, grid, s);
	}
}

// IWT coefficients of every launch frame into its work buffer (the model
// addressing of the launch), ahead of the encode kernel
static uint32_t run_iwt(struct airs_dev_engine *e, const struct airs_launch *L)
{
	IwtArgs a;
	memset(&a, 0, sizeof(a));
	a.src = (const uint8_t *)L->src;
	a.src_stride = L->src_stride;
	a.coef = (uint8_t *)L->model;
	a.coef_stride = L->model_stride;
	a.coef_ptrs = L->model_ptrs;
	a.coef_div = L->model_div ? L->model_div : 1u;
	a.frame_list = L->frame_list;
	a.frame_add = L->frame_add;
	a.frame_mul = L->frame_list ? 0u : L->frame_mul;
	a.n = L->n;
	const bool w2 = L->sample_bytes == 2;
	static bool attr_b = false;
	if (!attr_b) { // heads of frames up to 4 Mi samples: up to 128 KiB of LDS
		HIPCHECK(hipFuncSetAttribute((const void *)iwt_heads_b_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
					     (int)(AIRS_IWT_LDS_MAX * 2u)));
		attr_b = true;
	}
	// whole 64-sample blocks, 16-byte aligned frames and work buffers: the
	// register kernel
	const bool al = ((uintptr_t)L->src & 15u) == 0 && (L->src_stride & 15u) == 0 &&
			(L->model_ptrs ? L->model_ptrs_al16 != 0u
				       : ((uintptr_t)L->model & 15u) == 0 && (L->model_stride & 15u) == 0);
#ifndef AIRS_IWT_TWO_PHASE
#define AIRS_IWT_TWO_PHASE 1
#endif
	if (AIRS_IWT_TWO_PHASE && L->n % 64u == 0 && L->n >= 128u && L->n / 64u <= 65536u && al) {
		const uint32_t nb = L->n / 64u, wpf = (nb + IWT_RB - 1u) / IWT_RB;
		const uint64_t grid = (uint64_t)wpf * L->num_frames;
		if (grid > 0x7FFFFFFFull)
			return ERRV(E_PARAMS_INVALID);
		a.heads = (int16_t *)airs_dev_scratch(e, AIRS_NSLOT - 1, (size_t)nb * L->num_frames * 2u);
		if (!a.heads)
			return ERRV(E_GENERIC);
		if (w2)
			hipLaunchKernelGGL(iwt_blocks_a_kernel<2>, dim3((uint32_t)grid), dim3(256), 0, e->stream, a, wpf);
		else
			hipLaunchKernelGGL(iwt_blocks_a_kernel<4>, dim3((uint32_t)grid), dim3(256), 0, e->stream, a, wpf);
		const size_t lds = (size_t)((nb + 63u) & ~63u) * 2u;
		hipLaunchKernelGGL(iwt_heads_b_kernel, dim3(L->num_frames), dim3(64), lds, e->stream, a);
		HIPCHECK(hipGetLastError());
		return 0;
	}
	if (L->n % 64u == 0 && L->n >= 128u && L->n <= 65536u && al) {
		if (w2)
			hipLaunchKernelGGL(iwt_block_kernel<2>, dim3(L->num_frames), dim3(1024), 0, e->stream, a);
		else
			hipLaunchKernelGGL(iwt_block_kernel<4>, dim3(L->num_frames), dim3(1024), 0, e->stream, a);
		HIPCHECK(hipGetLastError());
		return 0;
	}
	if (L->n <= AIRS_IWT_LDS_MAX) {
		static bool attr = false;
		if (!attr) {
			const int mx = (int)(AIRS_IWT_LDS_MAX * 2u);
			HIPCHECK(hipFuncSetAttribute((const void *)iwt_frame_kernel<2>,
						     hipFuncAttributeMaxDynamicSharedMemorySize, mx));
			HIPCHECK(hipFuncSetAttribute((const void *)iwt_frame_kernel<4>,
						     hipFuncAttributeMaxDynamicSharedMemorySize, mx));
			attr = true;
		}

		const size_t lds = (size_t)((L->n + 63u) & ~63u) * 2u; // whole swizzle blocks
		if (w2)
			hipLaunchKernelGGL(iwt_frame_kernel<2>, dim3(L->num_frames), dim3(1024), lds, e->stream, a);
		else
			hipLaunchKernelGGL(iwt_frame_kernel<4>, dim3(L->num_frames), dim3(1024), lds, e->stream, a);
		HIPCHECK(hipGetLastError());
		return 0;
	}
	if (L->num_frames > 65535u)
		return ERRV(E_PARAMS_INVALID);
	const uint32_t cb = min((L->n + 255u) / 256u, 1024u);
	if (w2)
		hipLaunchKernelGGL(iwt_copy_kernel<2>, dim3(cb, L->num_frames), dim3(256), 0, e->stream, a);
	else
		hipLaunchKernelGGL(iwt_copy_kernel<4>, dim3(cb, L->num_frames), dim3(256), 0, e->stream, a);
	for (uint32_t st = 1; st < L->n; st <<= 1) {
		const uint32_t items = (uint32_t)(((uint64_t)L->n + 2ull * st - 1ull) / (2ull * st));
		const uint32_t gb = min((items + 255u) / 256u, 1024u);
		hipLaunchKernelGGL(iwt_level_kernel, dim3(gb, L->num_frames), dim3(256), 0, e->stream, a, st, 0u);
		hipLaunchKernelGGL(iwt_level_kernel, dim3(gb, L->num_frames), dim3(256), 0, e->stream, a, st, 1u);
	}
	HIPCHECK(hipGetLastError());
	return 0;
}

static uint32_t select_rice(struct airs_dev_engine *e, const void *src, uint64_t src_stride, uint32_t div,
			    const uint64_t *ptrs, uint32_t sample_bytes, uint32_t n, uint32_t num_frames,
			    const uint32_t *flist, uint32_t fadd, uint32_t fmul, uint32_t preprocessing, uint32_t *out_g);

extern "C" uint32_t airs_dev_encode(struct airs_dev_engine *e, const struct airs_launch *L)
{
	if (!e || !L || L->n == 0 || L->num_frames == 0)
		return ERRV(E_GENERIC);
	if (L->preprocessing > PRE_MODEL)
		return ERRV(E_PARAMS_INVALID);
	if (L->preprocessing == PRE_IWT && (L->model_mode == AIRS_MODEL_UPDATE ||
					    (!L->model && !L->model_ptrs)))
		return ERRV(E_PARAMS_INVALID);
	if (L->encoder_type > ENC_MULTI || (L->sample_bytes != 2 && L->sample_bytes != 4))
		return ERRV(E_PARAMS_INVALID);
	const uint32_t segn = seg_chunks(L->sample_bytes == 4 ? 4 : 2, L->model_mode ? 1 : 0) * AIRS_SEG;
	const uint32_t spf = (L->n + segn - 1) / segn;
	const uint64_t segs = (uint64_t)spf * L->num_frames;
	if (segs > 0x7FFFFFFFull)
		return ERRV(E_PARAMS_INVALID);
	uint32_t r = ensure_granules(e, (size_t)segs);
	if (r)
		return r;
	// CMP_GPU_AUTO_RICE: fused into the encode kernel for frames of a few
	// segments without a model; otherwise the sliced selection writes g first.
	// A fused segment waits at its frame's candidate barrier for LATER blocks
	// of its frame (spf of the 128 workgroup slots of its XCD): on an engine
	// that may share the GPU only frames of up to AUTO_SHARED_MAX_SPF segments,
	// so that a kernel on another stream would have to hold all but a few of
	// an XCD's slots to delay the barrier
	const uint32_t auto_spf_max = e->opt_exclusive ? AUTO_MAX_SPF : AUTO_SHARED_MAX_SPF;
	const bool auto_fused = L->auto_rice && L->encoder_type == ENC_ZERO &&
				L->model_mode == AIRS_MODEL_NONE &&
				(L->preprocessing == PRE_NONE || L->preprocessing == PRE_DIFF) && spf <= auto_spf_max;
	const uint32_t *frame_g = L->frame_g;
	bool iwt_done = false;
	if (L->auto_rice && !auto_fused && L->encoder_type == ENC_ZERO) {
		if (!L->frame_g_scratch || L->preprocessing == PRE_MODEL)
			return ERRV(E_GENERIC);
		if (L->preprocessing == PRE_IWT) {
			// IWT passes: the coefficients first, then the selection over them
			// (the IWT residual is the coefficient: NONE on 16-bit values)
			r = run_iwt(e, L);
			if (r)
				return r;
			iwt_done = true;
			r = select_rice(e, L->model, L->model_stride, L->model_div ? L->model_div : 1u, L->model_ptrs, 2u, L->n,
					L->num_frames, L->frame_list, L->frame_add, L->frame_list ? 0u : L->frame_mul, PRE_NONE,
					L->frame_g_scratch);
		} else {
			r = select_rice(e, L->src, L->src_stride, 1u, nullptr, L->sample_bytes, L->n, L->num_frames,
					L->frame_list, L->frame_add, L->frame_list ? 0u : L->frame_mul, L->preprocessing,
					L->frame_g_scratch);
		}
		if (r)
			return r;
		frame_g = L->frame_g_scratch;
	}
	if (auto_fused) {
		if (segs * 16u > e->ktot_cap) {
			HIPCHECK(hipStreamSynchronize(e->stream));
			(void)hipFree(e->ktot);
			e->ktot = nullptr;
			const size_t want = segs * 16u + segs * 8u + 16384u;
			HIPCHECK(hipMalloc(&e->ktot, want * sizeof(uint64_t)));
			HIPCHECK(hipMemset(e->ktot, 0, want * sizeof(uint64_t)));
			e->ktot_cap = want;
		}
	}

	KArgs k;
	memset(&k, 0, sizeof(k));
	k.src = (const uint8_t *)L->src;
	k.dst = (uint8_t *)L->dst;
	k.model = (uint8_t *)L->model;
	k.model_ptrs = L->model_ptrs;
	k.frame_list = L->frame_list;
	k.frame_g = frame_g;
	k.ktot = auto_fused ? e->ktot : nullptr;
	k.seqs = L->seqs;
	k.checksums = L->checksums;
	k.ids = L->ids;
	k.status = L->status;
	k.needed = L->needed;
	k.agg = e->agg;
	k.tail = e->tail;
	k.ticket = e->ticket;
	k.src_stride = L->src_stride;
	k.dst_stride = L->dst_stride;
	k.model_stride = L->model_stride;
	k.model_div = L->model_div ? L->model_div : 1u;
	k.frame_add = L->frame_add;
	k.frame_mul = L->frame_list ? 0u : L->frame_mul;
	k.id_base = L->id_base;
	k.id_step = L->id_step;
	k.fail_bit = L->fail_bit;
	k.n = L->n;
	k.segs_per_frame = spf;
	k.num_segs = (uint32_t)segs;
	k.cap = L->cap;
	k.g = L->encoder_param;
	k.outlier_param = L->outlier_param;
	k.model_mode = L->model_mode;
	k.model_rate = L->model_rate;
	k.is_unsigned = L->is_unsigned;
	k.checksum = L->checksum_enabled;
	k.seq = L->seq;
	k.pre_hdr = L->preprocessing;
	k.enc_hdr = L->encoder_type;
	k.model_rate_hdr = L->model_rate;
	k.ticket_base = e->ticket_base;
	k.img_words = image_words(L->encoder_type, (frame_g || auto_fused) ? 0u : L->encoder_param);
	k.epoch = next_epoch(e);
#if AIRS_ABLATE
	k.dbg = g_dbg;
	if (g_dbg & 65536) {
		if (e->dbgts_n < 8u * segs * g_dbgts_ring) {
			(void)hipFree(e->dbgts);
			e->dbgts_n = 8u * segs * g_dbgts_ring;
			if (hipMalloc(&e->dbgts, e->dbgts_n * 8u) != hipSuccess)
				return ERRV(E_GENERIC);
			HIPCHECK(hipMemset(e->dbgts, 0, e->dbgts_n * 8u));
		}
		if (g_dbgts_ring == 1u)
			HIPCHECK(hipMemsetAsync(e->dbgts, 0, 8u * segs * 8u, e->stream));
		k.dbgts = e->dbgts + 8u * segs * (g_dbgts_launch++ % g_dbgts_ring);
	}
#endif

	bool rice = frame_g != nullptr || auto_fused ||
		    (L->encoder_param && (L->encoder_param & (L->encoder_param - 1u)) == 0u);
	if (L->preprocessing == PRE_MODEL && L->model_mode != AIRS_MODEL_UPDATE)
		return ERRV(E_PARAMS_INVALID);
	if (L->preprocessing == PRE_IWT && !iwt_done) {
		r = run_iwt(e, L);
		if (r)
			return r;
	}
	// whole segments and 16-byte aligned frames (and models): the FULL kernel
	bool full = L->n % segn == 0u && ((uintptr_t)L->src & 15u) == 0u && (L->src_stride & 15u) == 0u;
	if (L->model_mode != AIRS_MODEL_NONE || L->preprocessing == PRE_IWT)
		full = full && (L->model_ptrs ? L->model_ptrs_al16 != 0u
					      : ((uintptr_t)L->model & 15u) == 0u && (L->model_stride & 15u) == 0u);
	// FULL model launches run the look-back after the packing (enc_kernel.h
	// LBC): only when no frame can stop early (no fail bit)
	if (L->model_mode != AIRS_MODEL_NONE)
		full = full && L->fail_bit == UINT64_MAX;
	{
		// fused Rice selection: whole groups of 8 frames (XCD-local frames)
		const uint32_t grid = auto_fused ? (L->num_frames + 7u) / 8u * 8u * spf : (uint32_t)segs;
		if (L->sample_bytes == 2)
			dispatch_pre<2>(k, L->preprocessing, L->encoder_type, rice, full, L->model_mode, grid, e->stream);
		else
			dispatch_pre<4>(k, L->preprocessing, L->encoder_type, rice, full, L->model_mode, grid, e->stream);
	}
	HIPCHECK(hipGetLastError());
	if (k.dbg & 4u)
		e->ticket_base += (uint32_t)segs;
	return 0;
}

// ---- MODEL streams in one launch (enc_walk.hip) ----------------------------

// segment-walk workgroups (of 4096 samples) below which the walk takes
// 2048-sample segments, 8 samples per lane: twice the workgroups and waves
// (cfg5s8: 512 -> 1024 workgroups, 2 -> 4 data waves per SIMD): 67.8-68.6
// against 70.0-70.8 us once direct launches stopped touching the ticket
// counter
#ifndef AIRS_WALK_HALF_BELOW
#define AIRS_WALK_HALF_BELOW 1024u
#endif
// contexts from which a batch of walk_ctx_samples()-sample frames takes the
// context walk (one workgroup per context) instead of the segment walk
#ifndef AIRS_WALK_CTX_MIN
#define AIRS_WALK_CTX_MIN 128u
#endif

// words of ONE of the context walk's two images (16384 samples of the
// longer-coded pass), or 0 when the batch does not take the context walk:
// frames of its size, enough contexts to fill the CUs, two images in the LDS
// (no_ctx: the engine's CMP_GPU_OPT_NO_CONTEXT_WALK; batches with the
// fallback on the chip need the context walk and ignore it)
static uint32_t ctx_walk_words(const struct airs_walk *w, bool no_ctx)
{
	const uint32_t mbp = code_max_bits(w->enc_p, w->g_p, w->outl_p);
	const uint32_t mbs = code_max_bits(w->enc_s, w->g_s, w->outl_s);
	const uint32_t mb = mbp > mbs ? mbp : mbs;
	const uint32_t cw = ((walk_ctx_samples() / 4u * mb / 32u + 8u) + 3u) & ~3u;
	if (no_ctx && !w->fb)
		return 0u;
	if (w->n == walk_ctx_samples() && w->num_ctx >= AIRS_WALK_CTX_MIN && (2u * cw + 4u) * 4u <= 150u * 1024u &&
	    walk_ctx_lds(cw, w->fpc) <= AIRS_LDS_BYTES)
		return cw;
	return 0u;
}

// words of one image of the segment walk (walk_seg_samples(half) samples of
// the longer-coded pass at its longest codeword, plus flush words)
static uint32_t seg_walk_words(const struct airs_walk *w, bool half)
{
	const uint32_t mbp = code_max_bits(w->enc_p, w->g_p, w->outl_p);
	const uint32_t mbs = code_max_bits(w->enc_s, w->g_s, w->outl_s);
	return ((walk_seg_samples(half) * (mbp > mbs ? mbp : mbs) / 32u + 8u) + 3u) & ~3u;
}

extern "C" int airs_dev_walk_supported(const struct airs_walk *w)
{
	if (!w || !w->n || w->n % AIRS_SEG || !w->num_ctx || !w->fpc || (w->sample_bytes != 2 && w->sample_bytes != 4))
		return 0;
	if ((w->pre_p != PRE_NONE && w->pre_p != PRE_DIFF) || !walk_rice(w->enc_p, w->g_p) ||
	    !walk_rice(w->enc_s, w->g_s) || w->model_rate > 16u)
		return 0;
	if (((uintptr_t)w->src & 15u) || (w->src_stride & 15u))
		return 0;
	if (!w->model_ptrs && (((uintptr_t)w->model & 15u) || (w->model_stride & 15u)))
		return 0;
	if (w->fb && (!w->draws || !w->seq_out || w->cap != w->raw_size || w->raw_size < 16u + 2u * w->n ||
		      !ctx_walk_words(w, false)))
		return 0;
	// the LDS of the launch the batch takes: the context walk, or the segment
	// walk at its larger segment (either size may be chosen)
	if (!ctx_walk_words(w, false) && walk_seg_lds(seg_walk_words(w, false), w->fpc) > AIRS_LDS_BYTES)
		return 0;
	const uint64_t segs = (uint64_t)w->num_ctx * (w->n / AIRS_SEG);
	return segs <= 0x7FFFFFFFull && segs * w->fpc <= 0x7FFFFFFFull;
}


extern "C" uint32_t airs_dev_walk(struct airs_dev_engine *e, struct airs_walk *w)
{
	if (!e || !airs_dev_walk_supported(w))
		return ERRV(E_PARAMS_INVALID);
	// the segment walk takes 2048-sample segments when 4096-sample ones would
	// leave fewer than four workgroups per CU (AIRS_WALK_HALF_BELOW)
	bool half = (uint64_t)w->num_ctx * (w->n / AIRS_SEG) < AIRS_WALK_HALF_BELOW;
	if (e->opt_walk_segment) // CMP_GPU_OPT_WALK_SEGMENT forces the segment size
		half = e->opt_walk_segment == 2048u;
	const uint32_t spf = w->n / walk_seg_samples(half);
	const uint64_t total = (uint64_t)w->num_ctx * w->fpc;
	uint32_t r = ensure_granules(e, (size_t)(total * spf));
	if (r)
		return r;
	WArgs k;
	memset(&k, 0, sizeof(k));
	k.src = (const uint8_t *)w->src;
	k.src_stride = w->src_stride;
	k.dst = (uint8_t *)w->dst;
	k.dst_stride = w->dst_stride;
	k.cap = w->cap;
	k.model = (uint8_t *)w->model;
	k.model_stride = w->model_stride;
	k.model_ptrs = w->model_ptrs;
	k.checksums = w->checksums;
	k.checksum = w->checksum_enabled ? 1u : 0u;
	k.ids = w->ids;
	k.id_base = w->id_base;
	k.id_cstep = w->id_cstep;
	k.id_astep = w->id_astep;
	k.seq0s = w->seq0s;
	k.seq0 = w->seq0;
	k.status = w->status;
	k.agg = e->agg;
	k.tail = e->tail;
	k.ticket = e->ticket;
	k.n = w->n;
	k.spf = spf;
	k.num_ctx = w->num_ctx;
	k.fpc = w->fpc;
	k.iters = w->iters;
	k.g_p = w->g_p;
	k.outl_p = w->outl_p;
	k.g_s = w->g_s;
	k.outl_s = w->outl_s;
	k.model_rate = w->model_rate;
	k.is_unsigned = w->is_unsigned;
	k.fb = w->fb ? 1u : 0u;
	k.raw_size = w->raw_size;
	k.draws = w->draws;
	k.seq_out = w->seq_out;
	// one image for a segment of the longer-coded of the two passes at its
	// longest codeword, plus flush words (cfg5's MULTI g = 8: 34 bits, 17 KiB;
	// sized for 48 bits, two-data-wave workgroups did not all fit the CUs)
	k.img_words = seg_walk_words(w, half);
	k.epoch = next_epoch(e);
	// one context per workgroup when the frames have its size, there are
	// enough contexts to fill the CUs, and two images fit the LDS
	{
		// (CMP_GPU_OPT_NO_CONTEXT_WALK only where the segment walk fits)
		const bool seg_fits = walk_seg_lds(seg_walk_words(w, false), w->fpc) <= AIRS_LDS_BYTES;
		const uint32_t cw = ctx_walk_words(w, e->opt_no_ctx_walk != 0u && seg_fits);
		if (cw) {
			WArgs kc = k;
			kc.img_words = cw;
			if (!walk_ctx_encode(kc, w->sample_bytes, w->pre_p, w->enc_p, true, w->enc_s, true, e->stream))
				return ERRV(E_PARAMS_INVALID);
			HIPCHECK(hipGetLastError());
			return 0;
		}
	}
	// the fallback runs in the context walk only
	if (w->fb)
		return ERRV(E_PARAMS_INVALID);
#if AIRS_ABLATE
	k.dbg = g_dbg;
	if (g_dbg & 65536) {
		const size_t need = 8u * (size_t)total * spf;
		if (e->dbgts_n < need) {
			(void)hipFree(e->dbgts);
			e->dbgts_n = need;
			if (hipMalloc(&e->dbgts, e->dbgts_n * 8u) != hipSuccess)
				return ERRV(E_GENERIC);
		}
		HIPCHECK(hipMemsetAsync(e->dbgts, 0, need * 8u, e->stream));
		k.dbgts = e->dbgts;
	}
#endif
	k.ticket_base = e->walk_ticket_base;
	const int wr = walk_encode(k, w->sample_bytes, w->pre_p, w->enc_p, true, w->enc_s, true, e->stream,
				   e->opt_exclusive != 0u);

	if (wr < 0)
		return ERRV(E_PARAMS_INVALID);
	HIPCHECK(hipGetLastError());
	if (wr == 0) // the launch took tickets
		e->walk_ticket_base += (uint32_t)(w->num_ctx * spf);
	return 0;
}

extern "C" uint32_t airs_dev_encode_stream(struct airs_dev_engine *e, const void *src, uint32_t sample_bytes,
					  uint32_t n, uint32_t preprocessing, uint32_t encoder_type,
					  uint32_t encoder_param, uint32_t outlier_param, void *dst, uint32_t cap,
					  uint32_t *status)
{
	if (!e || !src || !dst || !status || n == 0 || n > AIRS_STREAM_MAX)
		return ERRV(E_GENERIC);
	if ((preprocessing != PRE_NONE && preprocessing != PRE_DIFF) || encoder_type > ENC_MULTI ||
	    (sample_bytes != 2 && sample_bytes != 4))
		return ERRV(E_PARAMS_INVALID);
	const uint32_t segn = stream_segn(sample_bytes);
	const uint32_t spf = (n + segn - 1u) / segn;
	uint32_t r = ensure_granules(e, spf);
	if (r)
		return r;
	KArgs k;
	memset(&k, 0, sizeof(k));
	k.src = (const uint8_t *)src;
	k.dst = (uint8_t *)dst;
	k.status = status;
	k.agg = e->agg;
	k.tail = e->tail;
	k.ticket = e->ticket;
	k.model_div = 1u;
	k.frame_mul = 1u;
	k.n = n;
	k.segs_per_frame = spf;
	k.num_segs = spf;
	k.cap = cap;
	k.g = encoder_param;
	k.outlier_param = outlier_param;
	k.pre_hdr = preprocessing;
	k.enc_hdr = encoder_type;
	k.img_words = image_words(encoder_type, encoder_param);
	k.epoch = next_epoch(e);
	const bool rice = encoder_param && (encoder_param & (encoder_param - 1u)) == 0u;
	const bool full = n % segn == 0u && ((uintptr_t)src & 15u) == 0u;
	// 16-bit GOLOMB_ZERO with g = 2^k, k <= 7: the Rice/ZERO kernel
	if (AIRS_RICE && full && sample_bytes == 2 && encoder_type == ENC_ZERO && rice &&
	    rice_encode(k, preprocessing, e->stream, true)) {
		HIPCHECK(hipGetLastError());
		return 0;
	}
	stream_encode(k, sample_bytes, preprocessing, encoder_type, rice, full, spf, e->stream);
	HIPCHECK(hipGetLastError());
	return 0;
}

extern "C" uint32_t airs_dev_checksum(struct airs_dev_engine *e, const void *src, uint64_t src_stride,
				      uint32_t sample_bytes, uint32_t n, uint32_t num_frames,
				      const uint32_t *frame_list, uint32_t *out)
{
	if (!e || !n || !num_frames)
		return ERRV(E_GENERIC);
	dim3 grid((num_frames + 15) / 16);
	// two launches: ck_pre_kernel forms the stripes' x P2
	// products, ck_chain_kernel runs the serial accumulator chains
	const uint32_t stripes = 2u * n >= 16u ? n / 8u : 0u;
	const uint32_t S4 = (stripes + 3u) & ~3u;
	// whole groups of 16 frames x 4 chains
	// (at least one granule: frames under 8 samples have no stripes, and an
	// empty request would return a slot that was never allocated)
	uint32_t *Y = (uint32_t *)airs_dev_scratch(e, AIRS_NSLOT - 4, (size_t)grid.x * 64u * S4 * 4u + 16u);
	if (!Y)
		return ERRV(E_GENERIC);
	if (stripes) {
		const dim3 pg(grid.x, min((S4 / 4u + 15u) / 16u, 65535u));
		if (sample_bytes == 2)
			hipLaunchKernelGGL(ck_pre_kernel<2>, pg, dim3(256), 0, e->stream, (const uint8_t *)src, src_stride,
					   n, num_frames, frame_list, S4, Y);
		else
			hipLaunchKernelGGL(ck_pre_kernel<4>, pg, dim3(256), 0, e->stream, (const uint8_t *)src, src_stride,
					   n, num_frames, frame_list, S4, Y);
	}
	if (sample_bytes == 2)
		hipLaunchKernelGGL(ck_chain_kernel<2>, grid, dim3(64), 0, e->stream, (const uint8_t *)src, src_stride, n,
				   num_frames, frame_list, S4, (const uint32_t *)Y, out);
	else
		hipLaunchKernelGGL(ck_chain_kernel<4>, grid, dim3(64), 0, e->stream, (const uint8_t *)src, src_stride, n,
				   num_frames, frame_list, S4, (const uint32_t *)Y, out);
	HIPCHECK(hipGetLastError());
	return 0;
}

// the sliced selection over frame f at src + (f / div) * stride, or ptrs[j]
static uint32_t select_rice(struct airs_dev_engine *e, const void *src, uint64_t src_stride, uint32_t div,
			    const uint64_t *ptrs, uint32_t sample_bytes, uint32_t n, uint32_t num_frames,
			    const uint32_t *flist, uint32_t fadd, uint32_t fmul, uint32_t preprocessing, uint32_t *out_g)
{
	if (!e || !n || !num_frames || !div)
		return ERRV(E_GENERIC);
	const uint8_t *s = (const uint8_t *)src;
	if (num_frames > e->rhist_cap) {
		HIPCHECK(hipStreamSynchronize(e->stream));
		(void)hipFree(e->rhist);
		e->rhist = nullptr;
		e->rhist_cap = 0;
		HIPCHECK(hipMalloc(&e->rhist, (size_t)num_frames * RICE_HSTRIDE * 4u));
		e->rhist_cap = num_frames;
	}
	HIPCHECK(hipMemsetAsync(e->rhist, 0, (size_t)num_frames * RICE_HSTRIDE * 4u, e->stream));
	const dim3 grid(num_frames, (n + RICE_SLICE - 1u) / RICE_SLICE); // <= 16 chunks per workgroup
	if (grid.y > 65535u)
		return ERRV(E_PARAMS_INVALID);
	if (sample_bytes == 2) {
		if (preprocessing == PRE_DIFF)
			hipLaunchKernelGGL((select_rice_hist_kernel<2, PRE_DIFF>), grid, dim3(256), 0, e->stream, s, src_stride,
					   div, ptrs, n, flist, fadd, fmul, e->rhist, out_g);
		else
			hipLaunchKernelGGL((select_rice_hist_kernel<2, PRE_NONE>), grid, dim3(256), 0, e->stream, s, src_stride,
					   div, ptrs, n, flist, fadd, fmul, e->rhist, out_g);
	} else {
		if (preprocessing == PRE_DIFF)
			hipLaunchKernelGGL((select_rice_hist_kernel<4, PRE_DIFF>), grid, dim3(256), 0, e->stream, s, src_stride,
					   div, ptrs, n, flist, fadd, fmul, e->rhist, out_g);
		else
			hipLaunchKernelGGL((select_rice_hist_kernel<4, PRE_NONE>), grid, dim3(256), 0, e->stream, s, src_stride,
					   div, ptrs, n, flist, fadd, fmul, e->rhist, out_g);
	}
	HIPCHECK(hipGetLastError());
	return 0;
}

extern "C" uint32_t airs_dev_select_rice(struct airs_dev_engine *e, const void *src, uint64_t src_stride,
					 uint32_t sample_bytes, uint32_t n, uint32_t num_frames,
					 const uint32_t *flist, uint32_t fadd, uint32_t fmul, uint32_t preprocessing,
					 uint32_t *out_g)
{
	return select_rice(e, src, src_stride, 1u, nullptr, sample_bytes, n, num_frames, flist, fadd, fmul,
			   preprocessing, out_g);
}

extern "C" uint32_t airs_dev_fb_step(struct airs_dev_engine *e, const struct airs_fb_step *s)
{
	if (!e || !s || !s->num_ctx)
		return ERRV(E_GENERIC);
	hipLaunchKernelGGL(fb_step_kernel, dim3((s->num_ctx + 255u) / 256u), dim3(256), 0, e->stream, *s);
	HIPCHECK(hipGetLastError());
	return 0;
}

extern "C" uint32_t airs_dev_fb_copy(struct airs_dev_engine *e, const struct airs_fb_step *s)
{
	if (!e || !s || !s->num_ctx || s->prev < 0 || !s->n)
		return ERRV(E_GENERIC);
	// frames of the device exact mode passed the prologue's size checks
	// (2n <= 2^24 - 1, cmp_header.h), so y <= 4096 here
	if ((s->n + 2047u) / 2048u > 65535u)
		return ERRV(E_GENERIC);
	const dim3 grid(s->num_ctx, (s->n + 2047u) / 2048u);
	if (s->sample_bytes == 2)
		hipLaunchKernelGGL(fb_copy_kernel<2>, grid, dim3(256), 0, e->stream, *s);
	else
		hipLaunchKernelGGL(fb_copy_kernel<4>, grid, dim3(256), 0, e->stream, *s);
	HIPCHECK(hipGetLastError());
	return 0;
}

extern "C" uint32_t airs_dev_pack_frames(struct airs_dev_engine *e, const void *src, uint64_t src_stride,
					uint32_t max_frame_bytes, const uint32_t *sizes, uint32_t num_frames,
					uint32_t err_floor, void *out, uint64_t *offsets)
{
	if (!e || !src || !sizes || !out || !offsets || !num_frames || (src_stride & 7u) || ((uintptr_t)src & 7u) ||
	    ((uintptr_t)out & 7u))
		return ERRV(E_GENERIC);
	hipLaunchKernelGGL(pack_scan_kernel, dim3(1), dim3(1024), 0, e->stream, sizes, num_frames, err_floor, offsets);
	const uint32_t ny = (uint32_t)min((((uint64_t)max_frame_bytes + 7u) / 8u + 1023u) / 1024u, (uint64_t)65535u);
	hipLaunchKernelGGL(pack_copy_kernel, dim3(num_frames, ny ? ny : 1u), dim3(256), 0, e->stream,
			   (const uint8_t *)src, src_stride, sizes, err_floor, offsets, (uint8_t *)out);
	HIPCHECK(hipGetLastError());
	return 0;
}

extern "C" uint32_t airs_dev_synth(struct airs_dev_engine *e, void *dst, uint32_t sample_bytes, uint64_t seed,
				   uint32_t frame0, uint32_t n, uint32_t num_frames, uint64_t stride,
				   uint32_t W)
{
	if (!e || !n || !num_frames)
		return ERRV(E_GENERIC);
	uint32_t gx = (n + 255) / 256;
	if (gx > 1024)
		gx = 1024;
	dim3 grid(gx, num_frames);
	if (sample_bytes == 2)
		hipLaunchKernelGGL(synth_kernel<2>, grid, dim3(256), 0, e->stream, (uint8_t *)dst, seed, frame0, n,
				   stride, W);
	else
		hipLaunchKernelGGL(synth_kernel<4>, grid, dim3(256), 0, e->stream, (uint8_t *)dst, seed, frame0, n,
				   stride, W);
	HIPCHECK(hipGetLastError());
	return 0;
}

extern "C" uint32_t airs_dev_patch_ids(struct airs_dev_engine *e, void *dst, uint64_t dst_stride,
				       uint32_t num_frames, uint32_t frame_add, uint32_t frame_mul,
				       const uint64_t *ids, const uint32_t *status)
{
	if (!e || !num_frames)
		return 0;
	hipLaunchKernelGGL(patch_ids_kernel, dim3((num_frames + 255) / 256), dim3(256), 0, e->stream,
			   (uint8_t *)dst, dst_stride, num_frames, frame_add, frame_mul, ids, status);
	HIPCHECK(hipGetLastError());
	return 0;
}

__global__ void patch_ids_at_kernel(uint8_t *data, const uint64_t *offsets, const uint64_t *ids, uint64_t n)
{
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	uint8_t *p = data + offsets[i] + 8u;
	const uint64_t id = ids[i];
	for (int b = 0; b < 6; b++)
		p[b] = (uint8_t)(id >> (40 - 8 * b));
}

extern "C" uint32_t airs_dev_patch_ids_at(struct airs_dev_engine *e, void *data, const uint64_t *offsets,
					  const uint64_t *ids, uint64_t n)
{
	if (!e || !n)
		return 0;
	hipLaunchKernelGGL(patch_ids_at_kernel, dim3((uint32_t)((n + 255u) / 256u)), dim3(256), 0, e->stream,
			   (uint8_t *)data, offsets, ids, n);
	HIPCHECK(hipGetLastError());
	return 0;
}

extern "C" void *airs_dev_malloc(size_t bytes)
{
	void *p = nullptr;
	if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess)
		return nullptr;
	return p;
}

extern "C" void airs_dev_free(void *p)
{
	if (p)
		(void)hipFree(p);
}

extern "C" uint32_t airs_dev_h2d(struct airs_dev_engine *e, void *dst, const void *src, size_t bytes)
{
	if (!bytes)
		return 0;
	HIPCHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, e->stream));
	return 0;
}

extern "C" uint32_t airs_dev_d2h(struct airs_dev_engine *e, void *dst, const void *src, size_t bytes)
{
	if (!bytes)
		return 0;
	HIPCHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, e->stream));
	return 0;
}

extern "C" uint32_t airs_dev_d2d_rows(struct airs_dev_engine *e, void *dst, size_t dpitch, const void *src,
				      size_t spitch, size_t width, size_t rows)
{
	if (!width || !rows)
		return 0;
	if (dpitch == width && spitch == width)
		HIPCHECK(hipMemcpyAsync(dst, src, width * rows, hipMemcpyDeviceToDevice, e->stream));
	else
		HIPCHECK(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, hipMemcpyDeviceToDevice, e->stream));
	return 0;
}

extern "C" uint32_t airs_dev_memset(struct airs_dev_engine *e, void *dst, int v, size_t bytes)
{
	if (!bytes)
		return 0;
	HIPCHECK(hipMemsetAsync(dst, v, bytes, e->stream));
	return 0;
}

// the fault count into the engine's coherent host word, in stream order
__global__ void fault_copy_kernel(const uint32_t *ticket, volatile uint32_t *hco)
{
	hco[AIRS_HCO_FAULT] = ticket[AIRS_FAULT_WORD];
}

static uint32_t sync_wait(struct airs_dev_engine *e, bool waited);
extern "C" int airs_dev_commit_release(struct airs_dev_engine *e, uint32_t seq, const uint64_t *ids, uint32_t total);

extern "C" uint32_t airs_dev_sync(struct airs_dev_engine *e)
{
	// one round trip: the fault word travels with the stream (a kernel writes
	// it to coherent host memory) instead of a blocking copy after the wait
	hipLaunchKernelGGL(fault_copy_kernel, dim3(1), dim3(1), 0, e->stream, e->ticket, e->hco);
	HIPCHECK(hipGetLastError());
	return sync_wait(e, false);
}

extern "C" uint32_t airs_dev_commit_begin(struct airs_dev_engine *e, const uint32_t *status, uint32_t num_ctx,
					  uint32_t fpc, void *dst, uint64_t dst_stride, uint32_t *seq)
{
	if (num_ctx > AIRS_HCO_MAX_CTX)
		return ERRV(E_PARAMS_INVALID);
	*seq = ++e->hco_seq;
	e->commit_dst = dst;
	e->commit_dst_stride = dst_stride;
	e->commit_status = status;
	e->commit_total = num_ctx * fpc;
	hipLaunchKernelGGL(commit_kernel, dim3(1), dim3(256), 0, e->stream, status, num_ctx, fpc, e->ticket, e->hco, *seq,
			   (uint8_t *)dst, dst_stride, e->commit_ticks);
	HIPCHECK(hipGetLastError());
	return 0;
}

// The host polls the kernel's signal in coherent memory instead of waiting
// for the stream, whose wake-up is the larger part of a batch's round trip
// (bounded; then the stream wait, which also reports a failed launch, after
// the release so that the kernel is not left waiting)
extern "C" uint32_t airs_dev_commit_wait(struct airs_dev_engine *e, uint32_t seq, uint32_t num_ctx, uint8_t *flags)
{
	for (uint64_t i = 0; i < e->commit_polls; i++) { // ~ a second of polls
		if (e->hco[AIRS_HCO_SEQ] == seq) {
			// the previous commit kernel ran before this one: its acknowledgement is final
			commit_verify(e);
			const uint32_t faults = e->hco[AIRS_HCO_FAULT];
			memcpy(flags, (const void *)((const volatile uint8_t *)e->hco + AIRS_HCO_FLAGS), num_ctx);
			if (faults) {
				snprintf(g_err, sizeof(g_err), "%u look-back give-ups", faults);
				fprintf(stderr, "airscmp: internal error: %s\n", g_err);
				return ERRV(102u); /* CMP_ERR_INT_BITSTREAM: the caller releases, then airs_dev_sync clears */
			}
			return 0;
		}
		__builtin_ia32_pause();
	}
	(void)airs_dev_commit_release(e, seq, nullptr, 0u);
	const uint32_t r = sync_wait(e, false);
	if (r)
		return r;
	if (e->hco[AIRS_HCO_SEQ] != seq) {
		snprintf(g_err, sizeof(g_err), "commit kernel did not signal");
		return ERRV(E_GENERIC);
	}
	memcpy(flags, (const void *)((const volatile uint8_t *)e->hco + AIRS_HCO_FLAGS), num_ctx);
	return 0;
}

// Release the commit kernel of `seq`: 1 when it patches the identifiers
// (ids given: the engine checks the kernel's acknowledgement at the next
// stream wait or commit, and patches the headers itself if the kernel gave
// up waiting for this release), 0 when the caller must patch them
// (no ids, more than the block holds, or a second release of the same seq:
// commit_wait released it on its time-out, with mode 0).
extern "C" int airs_dev_commit_release(struct airs_dev_engine *e, uint32_t seq, const uint64_t *ids, uint32_t total)
{
	if (e->hco_released == seq)
		return 0;
	e->hco_released = seq;
	if (ids && total > AIRS_HCO_MAX_IDS)
		ids = nullptr;
	const uint32_t b = seq & 1u;
	if (ids && e->commit_ids_cap[b] < total) {
		if (e->commit_ids[b])
			(void)hipHostFree(e->commit_ids[b]);
		e->commit_ids[b] = nullptr;
		e->commit_ids_cap[b] = 0;
		if (hipHostMalloc((void **)&e->commit_ids[b], (size_t)total * 8u, hipHostMallocDefault) == hipSuccess)
			e->commit_ids_cap[b] = total;
		else
			ids = nullptr; // (the caller patches)
	}
	if (ids) {
		memcpy((void *)((volatile uint8_t *)e->hco + AIRS_HCO_IDS), ids, (size_t)total * 8u);
		memcpy(e->commit_ids[b], ids, (size_t)total * 8u);
		e->pend_seq = seq;
		e->pend_total = total;
		e->pend_buf = b;
		e->pend_dst = e->commit_dst;
		e->pend_dst_stride = e->commit_dst_stride;
		e->pend_status = e->commit_status;
	}
	e->hco[AIRS_HCO_MODE] = ids ? 1u : 0u;
	__atomic_thread_fence(__ATOMIC_SEQ_CST);
	e->hco[AIRS_HCO_GO] = seq;
	return ids ? 1 : 0;
}

// The pending release's acknowledgement, once its commit kernel has ended
// (after a stream wait, or once the next commit kernel has signalled): a
// kernel that gave up before the release came left the headers alone, so
// the identifiers are patched here (queued on the stream; sync_wait waits
// for it).  Returns 1 when a patch was queued.
static int commit_verify(struct airs_dev_engine *e)
{
	if (!e->pend_seq)
		return 0;
	const uint32_t seq = e->pend_seq, ack = e->hco[AIRS_HCO_ACK];
	e->pend_seq = 0u;
	if ((ack & ~1u) == ((seq & 0x7FFFFFFFu) << 1) && (ack & 1u))
		return 0;
	// (the next write of this buffer is release seq + 2, after this patch ran)
	hipLaunchKernelGGL(patch_ids_kernel, dim3((e->pend_total + 255u) / 256u), dim3(256), 0, e->stream,
			   (uint8_t *)e->pend_dst, e->pend_dst_stride, e->pend_total, 0u, 1u,
			   (const uint64_t *)e->commit_ids[e->pend_buf], e->pend_status);
	return hipGetLastError() == hipSuccess ? 1 : 0;
}

static uint32_t sync_wait(struct airs_dev_engine *e, bool waited)
{
	if (!waited)
		HIPCHECK(hipStreamSynchronize(e->stream));
	if (commit_verify(e)) // a commit kernel gave up: the headers patched from here
		HIPCHECK(hipStreamSynchronize(e->stream));
	const uint32_t faults = e->hco[AIRS_HCO_FAULT];
#if AIRS_ABLATE
	if ((g_dbg & 65536) && g_dbgts_path[0]) { // the debug timeline (scripts/ts_analyze.py)
		FILE *f = fopen(g_dbgts_path, "wb");
		if (f && e->dbgts) {
			uint64_t *h = (uint64_t *)malloc(e->dbgts_n * 8u);
			if (h && hipMemcpy(h, e->dbgts, e->dbgts_n * 8u, hipMemcpyDeviceToHost) == hipSuccess)
				fwrite(h, 8u, e->dbgts_n, f);
			free(h);
		}
		if (f)
			fclose(f);
	}
	if (g_dbg & 256) {
		uint32_t st[4];
		HIPCHECK(hipMemcpy(st, e->ticket + 20, sizeof(st), hipMemcpyDeviceToHost));
		fprintf(stderr, "airscmp look-back stats: lookbacks=%u rounds=%u retries=%u tail_repolls=%u\n", st[0],
			st[1], st[2], st[3]);
		(void)hipMemset(e->ticket + 20, 0, sizeof(st));
	}
#endif
	if (faults) {
		snprintf(g_err, sizeof(g_err), "%u look-back give-ups", faults);
		fprintf(stderr, "airscmp: internal error: %s\n", g_err);
		(void)hipMemset(e->ticket + AIRS_FAULT_WORD, 0, sizeof(faults));
		return ERRV(102u); /* CMP_ERR_INT_BITSTREAM */
	}
	return 0;
}
