// enc_common.h -- declarations and device helpers shared by the encode
// kernels (encode.hip: the general kernel and the device layer;
// enc_stream.hip: payload-only streams).  Reference citations as in encode.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "airs_dev.h"

#ifndef AIRS_WG
#define AIRS_WG 256
#endif
#define AIRS_PT 16
#define AIRS_SEG (AIRS_WG * AIRS_PT)
// encode kernel: EWG threads per workgroup, EPT samples per lane per chunk
// (EWG * EPT = AIRS_SEG samples per chunk)
#ifndef AIRS_EWG
#define AIRS_EWG 256
#endif
#define EWG AIRS_EWG
#define EPT (AIRS_SEG / AIRS_EWG)
// bounded spins: ~2^22 polls with s_sleep is far beyond any legitimate wait
#define AIRS_SPIN_LIMIT (1u << 22)
// engine->ticket[AIRS_FAULT_WORD] counts look-back give-ups (must stay 0)
#define AIRS_FAULT_WORD 16
// engine->ticket[AIRS_WALK_TICKET]: the segment walk's logical block tickets
#define AIRS_WALK_TICKET 32
// the engine's coherent page-locked block (kernels write it over the bus,
// the host polls it): words, per-context flags, identifiers
#define AIRS_HCO_FAULT 0          // word: the fault count (airs_dev_sync, the commit kernel)
#define AIRS_HCO_SEQ 1            // word: the commit kernel's signal (its sequence number)
#define AIRS_HCO_GO 2             // word: the host's release of that kernel (the same number)
#define AIRS_HCO_MODE 3           // word: 1 = patch the identifiers, 0 = not
#define AIRS_HCO_ACK 4            // word: the commit kernel's acknowledgement, written when it
                                  // has finished: (seq & 0x7FFFFFFF) << 1 | 1 if it patched
#define AIRS_HCO_FLAGS 64         // byte offset of the per-context flags
#define AIRS_HCO_MAX_CTX 8192u    // flags for up to this many contexts
#define AIRS_HCO_IDS (64u + 8192u) // byte offset of the identifiers
#define AIRS_HCO_BYTES 65536u     // block size
#define AIRS_HCO_MAX_IDS ((AIRS_HCO_BYTES - AIRS_HCO_IDS) / 8u)

// Ablation switches (AIRS_DBG bits, benchmarking only) are compiled in only
// with -DAIRS_ABLATE=1: in the product build every DBG() is a constant false,
// so the checks cost no instructions.
#ifndef AIRS_ABLATE
#define AIRS_ABLATE 0
#endif
#define DBG(bits) (AIRS_ABLATE && (a.dbg & (bits)))

#define ERRV(code) ((uint32_t)0u - (uint32_t)(code))
#define E_GENERIC 1u
#define E_PARAMS_INVALID 10u
#define E_DST_TOO_SMALL 30u
#define E_HDR_CMP_SIZE_TOO_LARGE 60u

namespace airs {

enum { PRE_NONE = 0, PRE_DIFF = 1, PRE_IWT = 2, PRE_MODEL = 3 };
enum { ENC_RAW = 0, ENC_ZERO = 1, ENC_MULTI = 2 };

struct KArgs {
	const uint8_t *src;
	uint8_t *dst;
	uint8_t *model;
	const uint64_t *model_ptrs;
	const uint32_t *frame_list;
	const uint32_t *frame_g;
	const uint32_t *checksums;
	const uint64_t *ids;
	uint32_t *status;
	uint32_t *needed;
	uint64_t *agg;   // per segment: (epoch<<1 | inclusive) << 32 | bits
	uint64_t *tail;  // per segment: epoch << 32 | last 32 bits of the segment's stream
	uint32_t *ticket;
	uint64_t src_stride, dst_stride, model_stride;
	uint32_t frame_add, frame_mul, model_div;
	uint32_t lbmode; // rice_kernel: bit 0 = every segment and its predecessors on one XCD (scalar look-back polls)
	uint64_t id_base, id_step, fail_bit;
	uint32_t n, segs_per_frame, num_segs, cap;
	uint32_t g, outlier_param;
	uint32_t model_mode, model_rate, is_unsigned, checksum;
	uint32_t seq, pre_hdr, enc_hdr, model_rate_hdr;
	uint32_t ticket_base, epoch;
	uint32_t img_words; // LDS image size: AIRS_SEG * (longest codeword) / 32 + 4, multiple of 4
	uint32_t dbg; // ablation switches (AIRS_DBG env, benchmarking only; 0 in production)
	uint64_t *dbgts; // AIRS_DBG bit 65536 (ablation builds): per-segment timeline
	// fused per-frame Rice selection (encode_kernel<..., AUTO>): per segment 16
	// granules, epoch << 32 | sum over its samples of min((m+1) >> k, 16), k = 0..15
	uint64_t *ktot;
	// per batch frame header sequence numbers (device-planned launches), else seq
	const uint8_t *seqs;
};

// frame_list entry of a launch position without a frame this launch
#define AIRS_NO_FRAME 0xFFFFFFFFu

// fused Rice selection: frames of at most AUTO_MAX_SPF segments (the frame's
// 16 * spf candidate granules are read by one wave in AUTO_MAX_SPF / 4 loads
// per lane); larger frames take the sliced selection (select_rice_hist_kernel) first
#ifndef AUTO_MAX_SPF
#define AUTO_MAX_SPF 32u
#endif
// ... on engines not marked CMP_GPU_OPT_EXCLUSIVE (the GPU may be shared)
#ifndef AUTO_SHARED_MAX_SPF
#define AUTO_SHARED_MAX_SPF 8u
#endif
// histogram bins: v = m + 1 in [1, 65536], bin = 8 floor(log2 v) + next 3 bits
#define AUTO_BINS 129u
// min(v >> k, 16) for every v of bin `bin` (top-bit position t = bin / 8, the
// three bits after it bin % 8): 16 when k <= t - 4, 0 when k > t, else the
// top t - k + 1 bits
__device__ __forceinline__ uint32_t auto_term(uint32_t bin, uint32_t k)
{
	const uint32_t t = bin >> 3, top4 = 8u + (bin & 7u);
	if (k + 4u <= t)
		return 16u;
	if (k > t)
		return 0u;
	return top4 >> (k + 3u - t);
}

// ---------------------------------------------------------------------
// Golomb coder constants (reference encoder.c:185-224, with
// golomb_upper_bound :63-110 and golomb_optimal_outlier_zero :154-182)
// ---------------------------------------------------------------------
struct Coder {
	uint32_t g, k, cutoff, outlier, magic;
};

template <int ENC>
__device__ __forceinline__ Coder make_coder(uint32_t g, uint32_t outlier_param)
{
	Coder c;
	c.g = g;
	c.k = 31u - (uint32_t)__clz((int)g);
	c.cutoff = (2u << c.k) - g;
	uint32_t limit = c.cutoff + (31u - c.k) * g;
	if (ENC == ENC_MULTI)
		limit = limit > 8u ? limit - 8u : 0u;
	uint64_t want = ENC == ENC_ZERO ? (uint64_t)c.cutoff + 16ull * g - 1ull : (uint64_t)outlier_param;
	c.outlier = (uint32_t)(want < limit ? want : limit);
	c.magic = g > 1u ? (uint32_t)((1ull << 32) / g) : 0xFFFFFFFFu;
	return c;
}

// Golomb codeword of v (reference encoder.c:303-324), len <= 32.
template <bool RICE>
__device__ __forceinline__ void golomb(uint32_t v, const Coder &c, uint32_t &cw, uint32_t &len)
{
	if (RICE) {
		// g = 2^k: q ones, a zero, k low bits; identical to the reference's
		// cutoff form because cutoff == g.
		uint32_t q = min(v >> c.k, 31u);
		len = q + c.k + 1u;
		cw = (((1u << q) - 1u) << (c.k + 1u)) | (v & (c.g - 1u));
	} else {
		uint32_t t = v - c.cutoff;
		uint32_t q = __umulhi(t, c.magic);
		uint32_t r = t - q * c.g;
		if (r >= c.g) {
			q += 1u;
			r -= c.g;
		}
		q = min(q, 31u);
		bool g0 = v < c.cutoff;
		len = g0 ? c.k + 1u : c.k + 2u + q;
		cw = g0 ? v : ((((1u << q) - 1u) << (c.k + 2u)) | (2u * c.cutoff + r));
	}
}

__device__ __forceinline__ uint32_t zigzag16(uint32_t u) // u: 16-bit residual pattern
{
	return ((u << 1) ^ (0u - ((u >> 15) & 1u))) & 0xFFFFu; // reference encoder.c:274-286
}

// v_bfm_b32: ((1 << w) - 1) << o, using the low 5 bits of w and o (no UB for
// the discarded escape lanes whose w is out of range)
__device__ __forceinline__ uint32_t bfm32(uint32_t w, uint32_t o)
{
	uint32_t r;
	asm("v_bfm_b32 %0, %1, %2" : "=v"(r) : "v"(w), "v"(o));
	return r;
}

// Mapped value (ZigZag, or the raw residual for UNCOMPRESSED) -> up to two
// (codeword, length) pieces (reference encoder.c:327-378).
template <int ENC, bool RICE>
__device__ __forceinline__ void code_from_m(uint32_t m, const Coder &c, uint32_t &cw1, uint32_t &l1,
					    uint32_t &cw2, uint32_t &l2)
{
	cw2 = 0u;
	l2 = 0u;
	if (ENC == ENC_RAW) {
		cw1 = m;
		l1 = 16u;
		return;
	}
	if (ENC == ENC_ZERO) {
		if (RICE) {
			// g = 2^k: v = m + 1, q = v >> k; the zero-escape length k+17 is
			// exactly the q = 16 case of k + 1 + q, so the length needs no select
			const uint32_t v = m + 1u, q = v >> c.k;
			l1 = c.k + 1u + min(q, 16u);
			cw1 = q > 16u ? m : (bfm32(q, c.k + 1u) | (v & (c.g - 1u)));
		} else {
			uint32_t gcw, glen;
			golomb<false>(m + 1u, c, gcw, glen);
			const bool esc = m >= c.outlier;
			cw1 = esc ? m : gcw; // zero codeword + 16 raw bits in one piece
			l1 = esc ? c.k + 17u : glen;
		}
		return;
	}
	const bool esc = m >= c.outlier;
	const uint32_t d = m - c.outlier;
	const uint32_t lvl = d < 4u ? 0u : (31u - (uint32_t)__clz((int)d)) >> 1;
	golomb<RICE>(esc ? c.outlier + lvl : m, c, cw1, l1);
	cw2 = esc ? d : 0u;
	l2 = esc ? 2u * (lvl + 1u) : 0u;
}

// code length only (the lengths pass)
template <int ENC, bool RICE>
__device__ __forceinline__ uint32_t len_from_m(uint32_t m, const Coder &c)
{
	if (ENC == ENC_RAW)
		return 16u;
	if (ENC == ENC_ZERO && RICE)
		return c.k + 1u + min((m + 1u) >> c.k, 16u);
	uint32_t cw1, l1, cw2, l2;
	code_from_m<ENC, RICE>(m, c, cw1, l1, cw2, l2);
	return l1 + l2;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t v)
{
	return __builtin_bswap32(v);
}

__device__ __forceinline__ uint64_t gran_load(const uint64_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void gran_store(uint64_t *p, uint64_t v)
{
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 16 samples of this lane: first sample index `first` inside the frame
// (vector loads when the frame base is 16-byte aligned: uniform per frame)
template <int W>
__device__ __forceinline__ void load16(const uint8_t *fsrc, uint32_t first, uint32_t n, uint32_t (&x)[AIRS_PT])
{
	if (first + AIRS_PT <= n && ((uintptr_t)fsrc & 15u) == 0) {
		if (W == 2) {
			const uint4 *p = reinterpret_cast<const uint4 *>(fsrc + (size_t)first * 2u);
			uint4 a = p[0], b = p[1];
			uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
			for (int j = 0; j < 8; j++) {
				x[2 * j] = w[j] & 0xFFFFu;
				x[2 * j + 1] = w[j] >> 16;
			}
		} else {
			const uint4 *p = reinterpret_cast<const uint4 *>(fsrc + (size_t)first * 4u);
#pragma unroll
			for (int q = 0; q < 4; q++) {
				uint4 a = p[q];
				x[4 * q + 0] = a.x & 0xFFFFu;
				x[4 * q + 1] = a.y & 0xFFFFu;
				x[4 * q + 2] = a.z & 0xFFFFu;
				x[4 * q + 3] = a.w & 0xFFFFu;
			}
		}
	} else {
#pragma unroll
		for (int j = 0; j < AIRS_PT; j++) {
			uint32_t i = first + j;
			uint32_t v = 0;
			if (i < n) {
				if (W == 2)
					v = reinterpret_cast<const uint16_t *>(fsrc)[i];
				else
					v = reinterpret_cast<const uint32_t *>(fsrc)[i] & 0xFFFFu;
			}
			x[j] = v;
		}
	}
}

__device__ __forceinline__ void load16_model(const uint8_t *m, uint32_t first, uint32_t n, uint32_t (&x)[AIRS_PT])
{
	load16<2>(m, first, n, x);
}

// Header dwords 0..4 of a frame (reference header.c:24-67), big-endian
// values; bytes 20-21 (outlier low half) travel with the first payload dword.
__device__ __forceinline__ void header_words(uint32_t (&h)[5], uint32_t size, uint32_t orig, uint64_t id,
					     uint32_t seq, uint32_t pre, uint32_t ck, uint32_t enc, uint32_t rate,
					     uint32_t par, uint32_t outl)
{
	h[0] = (0x8000u | 600u) << 16 | (size >> 8);
	h[1] = (size & 0xFFu) << 24 | (orig & 0xFFFFFFu);
	h[2] = (uint32_t)(id >> 16);
	h[3] = (uint32_t)(id & 0xFFFFu) << 16 | (seq & 0xFFu) << 8 | (pre << 4 | ck << 3 | enc);
	h[4] = (rate & 0xFFu) << 24 | (par & 0xFFFFu) << 8 | ((outl >> 16) & 0xFFu);
}

// DPP inclusive prefix sum over the 64 lanes of a wave (GFX9 row_shr +
// row_bcast sequence; no LDS traffic).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
	v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false); // row_shr:1
	v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false); // row_shr:2
	v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false); // row_shr:4
	v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false); // row_shr:8
	v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false); // row_bcast:15
	v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false); // row_bcast:31
	return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
	return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(v), 63);
}

// Two 16-bit lanes per VGPR (v_pk_* ops): samples, residuals and mapped
// values of a lane's 16 samples travel as 8 packed registers.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u16x2 pk(uint32_t x)
{
	return __builtin_bit_cast(u16x2, x);
}

__device__ __forceinline__ uint32_t unpk(u16x2 x)
{
	return __builtin_bit_cast(uint32_t, x);
}

__device__ __forceinline__ uint32_t half16(uint32_t w, uint32_t h)
{
	return h ? w >> 16 : w & 0xFFFFu;
}

// ZigZag of two 16-bit residuals at once (reference encoder.c:274-286)
__device__ __forceinline__ uint32_t zigzag_pk(uint32_t u)
{
	const u16x2 x = pk(u);
	return unpk((x << (u16x2)(1)) ^ __builtin_bit_cast(u16x2, __builtin_bit_cast(i16x2, x) >> (i16x2)(15)));
}

// MODEL update of a sample pair (reference cmp.c:120-142):
//   (model*rate + x*(16-rate)) >> 4 = model + ((x - model)*(16-rate) >> 4)
// exactly (16*model is a multiple of 16; >> is the floor).  x and model are
// sign-extended (i16) or zero-extended (u16); flip = 0x80008000 for i16 turns
// the signed difference into one of zero-extended halves (sext(v) =
// zext(v ^ 0x8000) - 0x8000), 0 for u16.  |x - model| < 2^17 and r1 <= 16, so
// the product fits a 24-bit multiply; only the low 16 bits are kept.
// The same on zero-extended halves (u16, or both operands flipped):
// (x - model) per half, 24-bit multiply, floor shift, add back.
__device__ __forceinline__ uint32_t model_update_zx(uint32_t x, uint32_t model, int32_t r1)
{
	const int32_t d0 = (int32_t)(x & 0xFFFFu) - (int32_t)(model & 0xFFFFu);
	const int32_t d1 = (int32_t)(x >> 16) - (int32_t)(model >> 16);
	const int32_t n0 = (int32_t)(model & 0xFFFFu) + (__mul24(d0, r1) >> 4);
	const int32_t n1 = (int32_t)(model >> 16) + (__mul24(d1, r1) >> 4);
	return __builtin_amdgcn_perm((uint32_t)n1, (uint32_t)n0, 0x05040100u);
}

// flip = 0x80008000 for i16, 0 for u16; the result is the model itself
// (flipping both operands and the result: (m ^ f) + t = (m + t) ^ f mod 2^16)
__device__ __forceinline__ uint32_t model_update_pk(uint32_t x, uint32_t model, uint32_t flip, int32_t r1)
{
	return model_update_zx(x ^ flip, model ^ flip, r1) ^ flip;
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;

// Bit packer into an LDS image.  `nb` is a bit position in the LDS address
// space: 8 * (byte address of the image) + (bit offset inside the image) - 32,
// so the word that holds the 32 bits preceding the pending ones is at byte
// address (nb >> 3) & ~3 (no base add per step) and nb mod 32 is the pending
// count.  acc holds (at least) the last 32 + (nb mod 32) bits.  Every put ORs
// those preceding 32 bits into their word: when a word just completed that is
// the new word, otherwise it is the previous word again (or zeros before the
// lane's first bit), which ORs nothing new.  So there is one ds_or per piece
// and no select or branch.
struct Packer {
	uint64_t acc;
	uint32_t nb;

	__device__ __forceinline__ void init(const uint32_t *image, uint32_t bit)
	{
		acc = 0u;
		// the low 32 bits of a generic LDS pointer are its LDS byte address
		nb = ((uint32_t)(uintptr_t)image << 3) + bit - 32u;
	}
	__device__ __forceinline__ void put(uint32_t cw, uint32_t len) // len <= 32, cw < 2^len
	{
		acc = (acc << len) | cw;
		nb += len;
		// v_alignbit uses nb mod 32
		lds_u32 *w = reinterpret_cast<lds_u32 *>((uintptr_t)((nb >> 3) & ~3u));
		__hip_atomic_fetch_or(w, __builtin_amdgcn_alignbit((uint32_t)(acc >> 32), (uint32_t)acc, nb),
				      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
	}
	__device__ __forceinline__ void flush()
	{
		if (nb & 31u) {
			lds_u32 *w = reinterpret_cast<lds_u32 *>((uintptr_t)(((nb >> 3) & ~3u) + 4u));
			__hip_atomic_fetch_or(w, (uint32_t)acc << (32u - (nb & 31u)), __ATOMIC_RELAXED,
					      __HIP_MEMORY_SCOPE_WORKGROUP);
		}
	}
};

// Rice/ZERO codeword table.  With v = m + 1 = q*2^k + low and q <= 16 the
// codeword is ((2^q - 1) << (k+1)) | low = v + 2^(q+k+1) - 2^(k+1) - q*2^k, so
// codeword = m + T'[q] with T'[q] = 2^(q+k+1) - 2^(k+1) - q*2^k + 1; every
// q >= 17 is the zero-escape, codeword m (T'[17] = 0), length k+17.
// Valid for k <= 11 (codewords < 2^29).
__device__ __forceinline__ uint2 rice_table_entry(uint32_t q, uint32_t k)
{
	if (q >= 17u)
		return make_uint2(0u, k + 17u);
	// (64-bit: q + k + 1 reaches 32 for k = 15; the entry itself wraps mod
	// 2^32, and cw = m + t stays exact since every codeword fits 32 bits)
	const uint32_t t = (uint32_t)((1ull << (q + k + 1u)) - (2ull << k) - ((uint64_t)q << k) + 1ull);
	return make_uint2(t, k + 1u + q);
}

// First look-back round's granule loads (wave 0, not the frame's first
// segment): LB_WIN windows of 64 aggregates, newest first, and the
// predecessor's tail.  Addresses are clamped into the frame instead of
// predicated, so the loads need no exec-mask branch (a predicated load made
// the compiler wait for it right away); the evaluation ignores the clamped
// lanes.
template <int LB_WIN>
__device__ __forceinline__ void lb_prefetch(const KArgs &a, uint64_t (&gv)[LB_WIN], uint64_t &tv0, uint32_t gseg,
					    uint32_t first_seg, uint32_t lane)
{
#pragma unroll
	for (int w = 0; w < LB_WIN; w++) {
		const int64_t idx = (int64_t)gseg - 1 - 64 * w - (int64_t)lane;
		gv[w] = gran_load(&a.agg[idx >= (int64_t)first_seg ? idx : (int64_t)first_seg]);
	}
	tv0 = gran_load(&a.tail[gseg - 1u]);
}

// all-ones when q > 16 (q < 2^16)
__device__ __forceinline__ uint32_t gt16_mask(uint32_t q)
{
	return (uint32_t)((int32_t)(16u - q) >> 31);
}

// Debug timeline (ablation builds, AIRS_DBG bit 65536): per segment, 8
// slots of the realtime clock (100 MHz): 0 start, 1 aggregate published,
// 2 look-back done, 3 look-back start, 4 segment done (wave 0); 5 look-back
// rounds | retries << 32, 6 tail re-polls; slot 7 = HW_ID << 32 | XCC_ID.  scripts/ts_analyze.py.
__device__ __forceinline__ void dbg_stamp(const KArgs &a, uint32_t gseg, uint32_t slot)
{
	if (DBG(131072u)) { // light timeline: slots 0 and 4 only, with the shader clock in 1 and 2
		if (DBG(65536u) && a.dbgts && threadIdx.x == 0 && (slot == 0 || slot == 4)) {
			uint64_t t, c;
			asm volatile("s_memrealtime %0\n s_memtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t), "=s"(c));
			a.dbgts[8u * gseg + slot] = t;
			a.dbgts[8u * gseg + (slot ? 2u : 1u)] = c;
			if (slot == 0) {
				uint32_t hw, xcc;
				asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
				asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
				a.dbgts[8u * gseg + 7u] = ((uint64_t)hw << 32) | xcc;
			}
		}
		return;
	}
	if (DBG(65536u) && a.dbgts && threadIdx.x == 0) {
		uint64_t t;
		asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t));
		a.dbgts[8u * gseg + slot] = t;
		if (slot == 0) {
			uint32_t hw, xcc;
			asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
			asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
			a.dbgts[8u * gseg + 7u] = ((uint64_t)hw << 32) | xcc;
		}
	}
}


// payload-only streams (enc_stream.hip): one frame of n <= AIRS_STREAM_MAX
// samples, no header; bit offsets stay below 2^32 at 48 bits per sample
uint32_t stream_segn(uint32_t sample_bytes);
// MODEL streams in one launch (enc_walk.hip, airs_walk in airs_dev.h)
struct WArgs {
	const uint8_t *src;
	uint8_t *dst;
	uint8_t *model;
	const uint64_t *model_ptrs;
	const uint32_t *checksums;
	const uint64_t *ids;
	const uint8_t *seq0s;
	uint32_t *status;
	uint64_t *agg;
	uint64_t *tail;
	uint32_t *ticket;
	uint64_t src_stride, dst_stride, model_stride;
	uint64_t id_base, id_cstep, id_astep;
	uint32_t n, spf, num_ctx, fpc;
	uint32_t cap, iters, seq0, epoch;
	uint32_t g_p, outl_p, g_s, outl_s;
	uint32_t model_rate, is_unsigned, checksum, img_words;
	uint32_t fb, raw_size; // uncompressed fallback on the chip (walk_ctx_kernel, airs_walk)
	uint32_t ticket_base;  // walk_kernel: ticket[AIRS_WALK_TICKET] before the launch
	uint32_t direct;       // walk_kernel: the whole grid is resident, logical index = block index
	uint32_t cus;          // walk_kernel: compute units of the device (direct launches: issue priority)
	uint8_t *draws;        // identifier draws per frame (fb)
	uint8_t *seq_out;      // sequence number per context after the walk (fb)
	uint32_t dbg;    // ablation builds: AIRS_DBG switches (0 in production)
	uint64_t *dbgts; // AIRS_DBG bit 65536: 8 realtime stamps per (workgroup, acquisition)
};
// the segment walk: < 0 no kernel for these passes; 0 launched with the
// ticket (the caller advances its ticket base); 1 launched direct
int walk_encode(const WArgs &k, uint32_t sample_bytes, uint32_t pre_p, uint32_t enc_p, bool rice_p, uint32_t enc_s,
		 bool rice_s, hipStream_t s, bool exclusive);
// one context per workgroup (frames of walk_ctx_samples() samples); img_words
// = words of ONE of its two 16384-sample images
bool walk_ctx_encode(const WArgs &k, uint32_t sample_bytes, uint32_t pre_p, uint32_t enc_p, bool rice_p,
		     uint32_t enc_s, bool rice_s, hipStream_t s);
uint32_t walk_ctx_samples();
// samples per segment of the segment walk (walk_kernel): 4096 with four data
// waves, 2048 with two (batches of few contexts); k.spf = n / that
uint32_t walk_seg_samples(bool half);
// the LDS bytes (dynamic + static) a walk launch takes, for the fit checks
// against the CU's 160 KiB before a batch is routed to it
size_t walk_ctx_lds(uint32_t img_words, uint32_t fpc);
size_t walk_seg_lds(uint32_t img_words, uint32_t fpc);
#define AIRS_LDS_BYTES (160u * 1024u)
// the Rice/ZERO frame kernel (enc_rice.hip): 16-bit NONE/DIFF, one g = 2^k
// (k <= 7), no model, whole 16 Ki-sample segments; false: not eligible
bool rice_encode(const KArgs &k, uint32_t pre, hipStream_t s, bool stream);
bool rice_auto_encode(const KArgs &k, uint32_t pre, hipStream_t s);
void stream_encode(const KArgs &k, uint32_t sample_bytes, uint32_t pre, uint32_t enc, bool rice, bool full,
		   uint32_t grid, hipStream_t s);

} // namespace airs
