// decode.hip -- MI355X (gfx950) decoder for AIRSPACE frames (SURVEY.md 8(f)
// row 1).  The reference has no decoder ("Decompression not implemented yet",
// programs/airspacecli.c:421-423); the format it inverts is the encoder's:
// header (lib/common/header.c:24-67), Golomb codewords (encoder.c:303-378),
// ZigZag (encoder.c:274-286) and the NONE / DIFF predictors
// (preprocess.c:250-290).  The CPU counterpart used as the test oracle is
// orc_decode (oracle/cmp_oracle.c).
//
// A Golomb stream has no index, so the payload of each frame is cut into
// subsequences of DEC_B bits and parsed in parallel by self-synchronisation.
// A workgroup owns DEC_WG consecutive subsequences, a DEC_WG * DEC_B bit
// span of the stream, which it stages in LDS with coalesced loads:
//   parse     thread s decodes codewords from a start (a guess: bit s*DEC_B)
//             until it passes (s+1)*DEC_B and records where it stopped (its
//             exit); inside the workgroup the starts are then settled in LDS
//             (thread s restarts from thread s-1's exit until none moves: a
//             wrong guess usually falls into step with the true parse after a
//             few codewords, so only the first threads redo any work)
//   rounds    the workgroup's first start is the previous workgroup's last
//             exit of the round before; rounds repeat until no workgroup's
//             last exit moves (workgroups whose first start is unchanged are
//             skipped)
//   scan      per frame, exclusive sum of the workgroups' symbol counts
//   output    each workgroup decodes its settled ranges again and writes the
//             residuals; DIFF / MODEL / IWT frames are inverted afterwards.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "airs_dev.h"

namespace airsdec {

#ifndef DEC_B
#define DEC_B 512u            // bits per subsequence
#endif
#define DEC_WG 256u           // subsequences (threads) per workgroup
#define DEC_SPANW (DEC_WG * DEC_B / 32u) // stream words a workgroup owns
#define DEC_HALO 8u           // words past the span (the last codeword and its window)
#define DEC_PRE 8u            // words before the span (the warm-up of the first range)
#ifndef DEC_WARM
#define DEC_WARM 192u         // bits decoded before a guessed start (speculative round; <= 32 * DEC_PRE)
#endif
#define DEC_BAD 0xFFFFFFFFu   // exit of a parse that met an invalid codeword
#define E_GENERIC 1u
#define E_PARAMS_INVALID 10u
#define E_INT_HDR 100u        // CMP_ERR_INT_HDR
#define E_INT_ENCODER 101u    // CMP_ERR_INT_ENCODER
#define E_INT_BITSTREAM 102u  // CMP_ERR_INT_BITSTREAM
#define ERRV(c) ((uint32_t)0u - (uint32_t)(c))
#define DEC_TILE 4096u        // samples per DIFF-scan tile

struct DecInfo {
	uint32_t n, nbits, hdr_bits, enc, pre, k, g, cutoff, outlier, nsub, wmax, status;
};

struct DecArgs {
	const uint8_t *src;
	uint64_t src_stride;
	uint32_t src_cap;
	uint32_t num_frames;
	uint16_t *dst;
	uint64_t dst_stride;
	uint32_t dst_samples;
	uint32_t *status;
	DecInfo *info;
	uint32_t *maxsub;
	uint32_t msub; // subsequences per frame allocated in the arrays below
	uint32_t mwg;  // workgroups per frame allocated in wg_cnt / wg_base
	uint32_t *exit_a, *exit_b, *cnt, *base, *changed;
	uint32_t *wg_cnt, *wg_base;
	uint16_t *tile_sum;
	const uint16_t *model; // MODEL frames: frame f's model at model + f * model_stride bytes
	uint64_t model_stride;
};

__device__ __forceinline__ uint32_t bswap32(uint32_t v)
{
	return __builtin_amdgcn_perm(v, v, 0x00010203u);
}

__device__ __forceinline__ uint32_t ilog2(uint32_t x)
{
	return 31u - __builtin_clz(x);
}

// one codeword at the top of the 64-bit window W: returns its length (0 =
// invalid) and m, the mapped value (UNCOMPRESSED: the raw 16 bits)
// RICE: the frame is GOLOMB_ZERO with g = 2^k (cutoff == g, so no extra
// bit, and q*g is a shift); chosen per frame, block-uniform
template <bool RICE>
__device__ __forceinline__ uint32_t dec_window(const DecInfo &I, uint64_t W, uint32_t &m)
{
	if (RICE) {
		const uint32_t q = (uint32_t)__clzll(~W);
		if (q > 32u)
			return 0u;
		uint32_t len = q + 1u + I.k;
		const uint32_t x = I.k ? (uint32_t)((W << (q + 1u)) >> (64u - I.k)) : 0u;
		const uint32_t u = (q << I.k) | x;
		if (u == 0u) {
			m = (uint32_t)((W << len) >> 48);
			len += 16u;
		} else {
			m = u - 1u;
		}
		return len > 48u ? 0u : len;
	}
	if (I.enc == 0u) { // UNCOMPRESSED (encoder.c:331-333)
		m = (uint32_t)(W >> 48);
		return 16u;
	}
	// Golomb (encoder.c:303-324): q ones, a zero, k bits (+1 past the cutoff)
	const uint32_t q = (uint32_t)__clzll(~W);
	if (q > 32u)
		return 0u;
	const uint64_t rest = W << (q + 1u);
	uint32_t x = I.k ? (uint32_t)(rest >> (64u - I.k)) : 0u;
	uint32_t len = q + 1u + I.k;
	if (x >= I.cutoff) {
		x = ((x << 1) | (uint32_t)((rest << I.k) >> 63)) - I.cutoff;
		len++;
	}
	const uint64_t u = (uint64_t)q * I.g + x;
	if (I.enc == 1u) { // GOLOMB_ZERO (encoder.c:335-351): 0 escapes 16 raw bits
		if (u == 0u) {
			m = (uint32_t)((W << len) >> 48);
			len += 16u;
		} else {
			m = (uint32_t)(u - 1u);
		}
	} else { // GOLOMB_MULTI (encoder.c:353-376)
		if (u < I.outlier) {
			m = (uint32_t)u;
		} else {
			const uint64_t lvl = u - I.outlier;
			if (lvl > 15u)
				return 0u;
			const uint32_t nb = 2u * ((uint32_t)lvl + 1u);
			if (len + nb > 64u)
				return 0u;
			m = I.outlier + (uint32_t)((W << len) >> (64u - nb));
			len += nb;
		}
	}
	return len > 48u ? 0u : len;
}

// Sequential bit reader over a workgroup's LDS copy of the stream (words
// already byte-swapped, so bit 31 of L[i] is the first): the next stream bits
// MSB-aligned in buf (nv valid, zeros below), refilled a word at a time.  A
// codeword that does not fit the valid bits (its decoded length exceeds nv:
// a bit it used past them was a fill zero) is decoded again from a full
// window read at its position.
template <bool RICE>
struct LdsReader {
	const uint32_t *L;
	uint32_t w0, w, nv, p; // L[0] holds stream word w0; next word; valid bits; payload bit position
	uint64_t buf;
	__device__ __forceinline__ uint64_t window(const DecInfo &I, uint32_t pos) const
	{
		const uint32_t abit = I.hdr_bits + pos, wi = (abit >> 5) - w0, o = abit & 31u;
		const uint64_t hi = ((uint64_t)L[wi] << 32) | L[wi + 1u];
		return o ? (hi << o) | (L[wi + 2u] >> (32u - o)) : hi;
	}
	__device__ __forceinline__ void init(const DecInfo &I, const uint32_t *l, uint32_t base_word, uint32_t pos)
	{
		L = l;
		w0 = base_word;
		p = pos;
		const uint32_t abit = I.hdr_bits + pos, wi = (abit >> 5) - w0, o = abit & 31u;
		buf = (((uint64_t)L[wi] << 32) | L[wi + 1u]) << o;
		nv = 64u - o;
		w = wi + 2u;
	}
	__device__ __forceinline__ uint32_t next(const DecInfo &I, uint32_t &m)
	{
		if (nv <= 32u) {
			buf |= (uint64_t)L[w] << (32u - nv);
			w++;
			nv += 32u;
		}
		uint32_t len = dec_window<RICE>(I, buf, m);
		if (len > nv || !len) {
			len = dec_window<RICE>(I, window(I, p), m); // slow path: the full window
			if (!len)
				return 0u;
			init(I, L, w0, p + len);
			return len;
		}
		buf = len < 64u ? buf << len : 0u;
		nv -= len;
		p += len;
		return len;
	}
};

// Stage workgroup wg's span of frame f's stream (with DEC_PRE words before
// it and DEC_HALO after) in LDS, byte-swapped; returns the stream word held
// in L[0].  Words outside the frame are clamped into it (their bits are never
// used by a valid parse).
#define DEC_LDSW (DEC_PRE + DEC_SPANW + DEC_HALO)
__device__ __forceinline__ uint32_t stage_span(const DecArgs &a, const DecInfo &I, uint32_t f, uint32_t wg,
					       uint32_t *L)
{
	const uint32_t *f32 = reinterpret_cast<const uint32_t *>(a.src + (uint64_t)f * a.src_stride);
	const int32_t w0 = (int32_t)((I.hdr_bits + wg * DEC_WG * DEC_B) >> 5) - (int32_t)DEC_PRE;
	for (uint32_t i = threadIdx.x; i < DEC_LDSW; i += DEC_WG)
		L[i] = bswap32(f32[min((uint32_t)max(w0 + (int32_t)i, 0), I.wmax)]);
	return (uint32_t)w0; // may be "negative": only differences are used
}

// header of every frame (header.c:24-67) -> DecInfo; NONE / DIFF frames only
__global__ void dec_hdr_kernel(DecArgs a)
{
	const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
	if (f >= a.num_frames)
		return;
	const uint8_t *b = a.src + (uint64_t)f * a.src_stride;
	DecInfo I;
	memset(&I, 0, sizeof(I));
	uint32_t st = 0;
	const uint32_t csize = ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 8) | b[4];
	const uint32_t osize = ((uint32_t)b[5] << 16) | ((uint32_t)b[6] << 8) | b[7];
	const uint32_t version = ((uint32_t)(b[0] & 0x7Fu) << 8) | b[1];
	I.pre = b[15] >> 4;
	const uint32_t ck = (b[15] >> 3) & 1u;
	I.enc = b[15] & 7u;
	const bool ext = !(I.pre == 0u && I.enc == 0u);
	const uint32_t hs = ext ? 22u : 16u;
	if (a.src_cap < 16u || !(b[0] >> 7) || version != 600u || csize > a.src_cap || csize < hs + (ck ? 4u : 0u) ||
	    (osize & 1u))
		st = ERRV(E_INT_HDR);
	else if (I.pre > 3u) // no such preprocessing (cmp.h: NONE, DIFF, IWT, MODEL)
		st = ERRV(E_INT_HDR);
	else if (I.pre == 3u && !a.model) // MODEL without its model
		st = ERRV(E_PARAMS_INVALID);
	else if (I.enc > 2u)
		st = ERRV(E_INT_ENCODER);
	I.n = osize / 2u;
	if (!st && I.n > a.dst_samples)
		st = ERRV(E_GENERIC);
	if (!st && I.enc != 0u) {
		const uint32_t g = ((uint32_t)b[17] << 8) | b[18];
		if (g == 0u) {
			st = ERRV(E_INT_ENCODER);
		} else {
			I.g = g;
			I.k = ilog2(g);
			I.cutoff = (2u << I.k) - g;
			I.outlier = ((uint32_t)b[19] << 16) | ((uint32_t)b[20] << 8) | b[21];
		}
	}
	if (!st) {
		I.hdr_bits = 8u * hs;
		I.nbits = 8u * (csize - hs - (ck ? 4u : 0u));
		I.wmax = min((csize + 3u) / 4u, a.src_cap / 4u) - 1u;
		I.nsub = I.n ? (I.nbits + DEC_B - 1u) / DEC_B : 0u;
		if (I.n && !I.nsub)
			st = ERRV(E_INT_BITSTREAM);
	}
	I.status = st;
	if (st)
		I.nsub = 0;
	a.info[f] = I;
	atomicMax(a.maxsub, I.nsub);
	if (!st && I.pre == 2u)
		atomicOr(a.maxsub + 2, 1u); // some frame needs the inverse IWT
}

// decode [start, end) of the stream from LDS: exit position and codeword count
template <bool RICE>
__device__ __forceinline__ uint32_t parse_range(const DecInfo &I, const uint32_t *L, uint32_t w0, uint32_t start,
						uint32_t end, uint32_t &cnt)
{
	cnt = 0;
	if (start == DEC_BAD)
		return DEC_BAD;
	uint32_t p = start;
	if (p < end) {
		LdsReader<RICE> br;
		br.init(I, L, w0, start);
		while (p < end) {
			uint32_t m;
			const uint32_t len = br.next(I, m);
			if (!len)
				return DEC_BAD;
			p += len;
			cnt++;
		}
	}
	return p;
}

// Speculative start of range r0 (> 0): decode from DEC_WARM bits before it
// and take the first codeword boundary at or past r0.  A Golomb parse falls
// into step with the true one within a few codewords, so this is almost
// always where the previous range's parse stops, and the settle pass finds
// nothing to redo.  DEC_BAD if an invalid codeword came first.
template <bool RICE>
__device__ __forceinline__ uint32_t warm_start(const DecInfo &I, const uint32_t *L, uint32_t w0, uint32_t r0)
{
	uint32_t p = r0 - min(r0, DEC_WARM);
	LdsReader<RICE> br;
	br.init(I, L, w0, p);
	while (p < r0) {
		uint32_t m;
		const uint32_t len = br.next(I, m);
		if (!len)
			return r0; // garbage before r0: guess r0 itself
		p += len;
	}
	return p;
}

// One parse round over workgroup-sized spans (grid: workgroups x frames).
// first: the speculative round (every start a guess).  Later rounds redo a
// workgroup only when its first start (the previous workgroup's last exit of
// the round before) moved, and inside it only the threads whose start moved.
template <bool RICE>
__device__ __forceinline__ void parse_wg(const DecArgs &a, const DecInfo &I, const uint32_t *exit_in,
					 uint32_t *exit_out, uint32_t first, uint32_t *L, uint32_t *s_exit, uint32_t *s_sum)
{
	const uint32_t f = blockIdx.y, wg = blockIdx.x, t = threadIdx.x, s = wg * DEC_WG + t;
	const bool live = s < I.nsub;
	const size_t o = (size_t)f * a.msub + s, o0 = (size_t)f * a.msub + wg * DEC_WG;
	uint32_t in_start = wg == 0u ? 0u : first ? 0u : exit_in[o0 - 1u];
	if (!first && a.base[o0] == in_start) { // block-uniform: nothing moved
		if (live)
			exit_out[o] = exit_in[o];
		return;
	}
	const uint32_t w0 = stage_span(a, I, f, wg, L);
	__syncthreads();
	if (first && wg) // the first range's start is a warm guess as well
		in_start = warm_start<RICE>(I, L, w0, wg * DEC_WG * DEC_B);
	const uint32_t end = min((s + 1u) * DEC_B, I.nbits);
	uint32_t start, ex = 0, c = 0;
	if (first) {
		start = t == 0u && wg == 0u ? 0u : live ? warm_start<RICE>(I, L, w0, s * DEC_B) : 0u;
		if (live)
			ex = parse_range<RICE>(I, L, w0, start, end, c);
	} else {
		// last round's result stands unless the start moves
		start = t == 0u ? in_start : a.base[o];
		if (live) {
			if (t == 0u) {
				ex = parse_range<RICE>(I, L, w0, start, end, c);
			} else {
				ex = exit_in[o];
				c = a.cnt[o];
			}
		}
	}
	for (;;) { // settle: thread t starts where thread t-1 stopped
		s_exit[t] = ex;
		__syncthreads();
		const uint32_t ns = t == 0u ? in_start : s_exit[t - 1u];
		const bool moved = live && ns != start;
		if (moved) {
			start = ns;
			ex = parse_range<RICE>(I, L, w0, start, end, c);
		}
		if (!__syncthreads_or(moved))
			break;
	}
	if (live) {
		if (!first && ex != exit_in[o] && (t + 1u == DEC_WG || s + 1u == I.nsub))
			*a.changed = 1u; // the next workgroup's first start moved
		exit_out[o] = ex;
		a.cnt[o] = c;
		a.base[o] = start;
	}
	// the workgroup's codeword count
	uint32_t v = live ? c : 0u;
	for (uint32_t d = 32; d; d >>= 1)
		v += __shfl_down(v, d, 64);
	if ((t & 63u) == 0u)
		s_sum[t >> 6] = v;
	__syncthreads();
	if (t == 0u) {
		uint32_t tot = 0;
		for (uint32_t w = 0; w < DEC_WG / 64u; w++)
			tot += s_sum[w];
		a.wg_cnt[(size_t)f * a.mwg + wg] = tot;
	}
}

__global__ __launch_bounds__(DEC_WG) void dec_parse_kernel(DecArgs a, const uint32_t *exit_in, uint32_t *exit_out,
							   uint32_t first)
{
	__shared__ uint32_t L[DEC_LDSW];
	__shared__ uint32_t s_exit[DEC_WG];
	__shared__ uint32_t s_sum[DEC_WG / 64u];
	const DecInfo I = a.info[blockIdx.y];
	if (blockIdx.x * DEC_WG >= I.nsub) // block-uniform
		return;
	if (I.enc == 1u && I.cutoff == I.g)
		parse_wg<true>(a, I, exit_in, exit_out, first, L, s_exit, s_sum);
	else
		parse_wg<false>(a, I, exit_in, exit_out, first, L, s_exit, s_sum);
}

// per frame: exclusive scan of the workgroups' codeword counts (one workgroup)
__global__ __launch_bounds__(1024) void dec_scan_kernel(DecArgs a)
{
	__shared__ uint32_t s_w[16];
	__shared__ uint32_t s_carry;
	const uint32_t f = blockIdx.x, t = threadIdx.x, lane = t & 63u, wid = t >> 6;
	const DecInfo I = a.info[f];
	const uint32_t nwg = (I.nsub + DEC_WG - 1u) / DEC_WG;
	if (t == 0)
		s_carry = 0;
	__syncthreads();
	for (uint32_t b0 = 0; b0 < nwg; b0 += 1024u) {
		const uint32_t i = b0 + t;
		const size_t o = (size_t)f * a.mwg + i;
		const uint32_t v = i < nwg ? a.wg_cnt[o] : 0u;
		uint32_t inc = v;
		for (uint32_t d = 1; d < 64u; d <<= 1) {
			const uint32_t y = __shfl_up(inc, d, 64);
			if (lane >= d)
				inc += y;
		}
		if (lane == 63u)
			s_w[wid] = inc;
		__syncthreads();
		uint32_t woff = s_carry;
		for (uint32_t w = 0; w < wid; w++)
			woff += s_w[w];
		if (i < nwg)
			a.wg_base[o] = woff + inc - v;
		__syncthreads();
		if (t == 1023u)
			s_carry = woff + inc;
		__syncthreads();
	}
	if (t == 0 && !I.status && s_carry < I.n) {
		// fewer than n codewords before the payload ends or an invalid one
		// (a parse that meets one stops, and every later range then starts
		// nowhere and counts nothing)
		a.info[f].status = ERRV(E_INT_BITSTREAM);
	}
}

// residuals (ZigZag undone) into dst; DIFF frames are summed afterwards
template <bool RICE>
__device__ __forceinline__ void out_wg(const DecArgs &a, const DecInfo &I, const uint32_t *exits, uint32_t *L,
				       uint32_t *s_w)
{
	const uint32_t f = blockIdx.y, wg = blockIdx.x, t = threadIdx.x, s = wg * DEC_WG + t, lane = t & 63u,
		       wid = t >> 6;
	const bool live = s < I.nsub;
	const size_t o = (size_t)f * a.msub + s;
	const uint32_t w0 = stage_span(a, I, f, wg, L);
	// this thread's first output index: the workgroup's base + its prefix
	const uint32_t v = live ? a.cnt[o] : 0u;
	uint32_t inc = v;
	for (uint32_t d = 1; d < 64u; d <<= 1) {
		const uint32_t y = __shfl_up(inc, d, 64);
		if (lane >= d)
			inc += y;
	}
	if (lane == 63u)
		s_w[wid] = inc;
	__syncthreads(); // also: the span is staged
	uint32_t b0 = a.wg_base[(size_t)f * a.mwg + wg] + inc - v;
	for (uint32_t w = 0; w < wid; w++)
		b0 += s_w[w];
	if (!live)
		return;
	uint32_t p = s ? exits[o - 1u] : 0u, j = b0;
	const uint32_t end = min((s + 1u) * DEC_B, I.nbits);
	uint16_t *out = a.dst + (uint64_t)f * (a.dst_stride / 2u);
	// samples are shifted into a 128-bit register and leave as 16-byte stores
	// of 8 (their run is contiguous; each lane's run starts anywhere), with
	// 2-byte stores for the unaligned ends
	const bool vec = (((uintptr_t)out | a.dst_stride) & 15u) == 0;
	uint64_t lo = 0, hi = 0;
	LdsReader<RICE> br;
	if (p < end)
		br.init(I, L, w0, p);
	while (p < end && j < I.n) {
		uint32_t m;
		const uint32_t len = br.next(I, m);
		if (!len)
			break;
		p += len;
		const uint32_t r = (I.enc == 0u ? m : ((m >> 1) ^ (0u - (m & 1u)))) & 0xFFFFu;
		if (!vec) {
			out[j++] = (uint16_t)r;
			continue;
		}
		lo = (lo >> 16) | (hi << 48);
		hi = (hi >> 16) | ((uint64_t)r << 48);
		if ((j & 7u) == 7u && j - 7u >= b0) {
			*reinterpret_cast<uint4 *>(out + (j - 7u)) =
				make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
		} else if ((j & 7u) == 7u) {
			// the run's first, partial group of 8: its own samples only
			for (uint32_t i = b0; i <= j; i++) {
				const uint32_t sh = 16u * (7u - (j - i)); // bit offset of sample i in (hi:lo)
				out[i] = (uint16_t)(sh >= 64u ? hi >> (sh - 64u) : lo >> sh);
			}
		}
		j++;
	}
	if (vec && (j & 7u)) { // the last, partial group
		const uint32_t g0 = max(j & ~7u, b0);
		for (uint32_t i = g0; i < j; i++) {
			const uint32_t sh = 16u * (8u - (j - i)); // bit offset of sample i in (hi:lo)
			out[i] = (uint16_t)(sh >= 64u ? hi >> (sh - 64u) : lo >> sh);
		}
	}
}

__global__ __launch_bounds__(DEC_WG) void dec_out_kernel(DecArgs a, const uint32_t *exits)
{
	__shared__ uint32_t L[DEC_LDSW];
	__shared__ uint32_t s_w[DEC_WG / 64u];
	const DecInfo I = a.info[blockIdx.y];
	if (blockIdx.x * DEC_WG >= I.nsub || I.status) // block-uniform
		return;
	if (I.enc == 1u && I.cutoff == I.g)
		out_wg<true>(a, I, exits, L, s_w);
	else
		out_wg<false>(a, I, exits, L, s_w);
}

// DIFF (preprocess.c:284-290) inverse: x[i] = x[i-1] + r[i] (int16 wrap), a
// three-step scan: tile sums, per-frame tile prefix, tile scans
__global__ __launch_bounds__(256) void dec_tile_sum_kernel(DecArgs a, uint32_t tiles)
{
	__shared__ uint32_t s_w[4];
	const uint32_t f = blockIdx.y, tile = blockIdx.x, t = threadIdx.x;
	const DecInfo I = a.info[f];
	if (I.status || I.pre != 1u || tile * DEC_TILE >= I.n)
		return;
	const uint16_t *x = a.dst + (uint64_t)f * (a.dst_stride / 2u) + (size_t)tile * DEC_TILE;
	const uint32_t cnt = min(DEC_TILE, I.n - tile * DEC_TILE);
	uint32_t sum = 0;
	if (cnt == DEC_TILE && (((uintptr_t)x) & 15u) == 0) {
		const uint4 *x4 = reinterpret_cast<const uint4 *>(x);
		for (uint32_t q = t; q < DEC_TILE / 8u; q += 256u) {
			const uint4 v = x4[q];
			sum += (v.x & 0xFFFFu) + (v.x >> 16) + (v.y & 0xFFFFu) + (v.y >> 16) + (v.z & 0xFFFFu) + (v.z >> 16) +
			       (v.w & 0xFFFFu) + (v.w >> 16);
		}
	} else {
		for (uint32_t i = t; i < cnt; i += 256u)
			sum += x[i];
	}
	for (uint32_t d = 32; d; d >>= 1)
		sum += __shfl_down(sum, d, 64);
	if ((t & 63u) == 0)
		s_w[t >> 6] = sum;
	__syncthreads();
	if (t == 0)
		a.tile_sum[(size_t)f * tiles + tile] = (uint16_t)(s_w[0] + s_w[1] + s_w[2] + s_w[3]);
}

// exclusive scan of a frame's tile sums (one workgroup per frame)
__global__ __launch_bounds__(1024) void dec_tile_prefix_kernel(DecArgs a, uint32_t tiles)
{
	__shared__ uint32_t s_w[16];
	__shared__ uint32_t s_carry;
	const uint32_t f = blockIdx.x, t = threadIdx.x, lane = t & 63u, wid = t >> 6;
	const DecInfo I = a.info[f];
	if (I.status || I.pre != 1u)
		return;
	const uint32_t nt = (I.n + DEC_TILE - 1u) / DEC_TILE;
	if (t == 0)
		s_carry = 0;
	__syncthreads();
	for (uint32_t b0 = 0; b0 < nt; b0 += 1024u) {
		const uint32_t i = b0 + t;
		uint16_t *ts = a.tile_sum + (size_t)f * tiles;
		const uint32_t v = i < nt ? ts[i] : 0u;
		uint32_t inc = v;
		for (uint32_t d = 1; d < 64u; d <<= 1) {
			const uint32_t y = __shfl_up(inc, d, 64);
			if (lane >= d)
				inc += y;
		}
		if (lane == 63u)
			s_w[wid] = inc;
		__syncthreads();
		uint32_t woff = s_carry;
		for (uint32_t w = 0; w < wid; w++)
			woff += s_w[w];
		if (i < nt)
			ts[i] = (uint16_t)(woff + inc - v);
		__syncthreads();
		if (t == 1023u)
			s_carry = woff + inc;
		__syncthreads();
	}
}

__global__ __launch_bounds__(256) void dec_tile_scan_kernel(DecArgs a, uint32_t tiles)
{
	__shared__ uint32_t s_w[4];
	const uint32_t f = blockIdx.y, tile = blockIdx.x, t = threadIdx.x, lane = t & 63u, wid = t >> 6;
	const DecInfo I = a.info[f];
	if (I.status || I.pre != 1u || tile * DEC_TILE >= I.n)
		return;
	uint16_t *x = a.dst + (uint64_t)f * (a.dst_stride / 2u) + (size_t)tile * DEC_TILE;
	const uint32_t cnt = min(DEC_TILE, I.n - tile * DEC_TILE);
	// thread t owns 16 consecutive samples
	uint32_t v[16], loc = 0;
	const bool vec = cnt == DEC_TILE && (((uintptr_t)x) & 15u) == 0;
	if (vec) {
		const uint4 *x4 = reinterpret_cast<const uint4 *>(x) + 2u * t;
		const uint4 p0 = x4[0], p1 = x4[1];
		const uint32_t w[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
		for (uint32_t q = 0; q < 8u; q++) {
			v[2 * q] = w[q] & 0xFFFFu;
			v[2 * q + 1] = w[q] >> 16;
		}
	} else {
#pragma unroll
		for (uint32_t j = 0; j < 16u; j++) {
			const uint32_t i = 16u * t + j;
			v[j] = i < cnt ? x[i] : 0u;
		}
	}
#pragma unroll
	for (uint32_t j = 0; j < 16u; j++)
		loc += v[j];
	uint32_t inc = loc;
	for (uint32_t d = 1; d < 64u; d <<= 1) {
		const uint32_t y = __shfl_up(inc, d, 64);
		if (lane >= d)
			inc += y;
	}
	if (lane == 63u)
		s_w[wid] = inc;
	__syncthreads();
	uint32_t run = a.tile_sum[(size_t)f * tiles + tile] + inc - loc;
	for (uint32_t w = 0; w < wid; w++)
		run += s_w[w];
#pragma unroll
	for (uint32_t j = 0; j < 16u; j++) {
		run += v[j];
		v[j] = run & 0xFFFFu;
	}
	if (vec) {
		uint4 *x4 = reinterpret_cast<uint4 *>(x) + 2u * t;
		x4[0] = make_uint4(v[0] | v[1] << 16, v[2] | v[3] << 16, v[4] | v[5] << 16, v[6] | v[7] << 16);
		x4[1] = make_uint4(v[8] | v[9] << 16, v[10] | v[11] << 16, v[12] | v[13] << 16, v[14] | v[15] << 16);
	} else {
#pragma unroll
		for (uint32_t j = 0; j < 16u; j++)
			if (16u * t + j < cnt)
				x[16u * t + j] = (uint16_t)v[j];
	}
}

// IWT inverse (preprocess.c:140-221 run backwards): the levels from the
// largest stride down; in each, the even coefficients are undone first (from
// their odd neighbours, which the forward even step read), then the odd ones
// (from the restored even neighbours).  Same int32 intermediates and int16
// wrap as the forward transform, so it is exact.
template <typename P>
__device__ __forceinline__ void iiwt_evens(P y, uint32_t n, uint32_t s, uint32_t t0, uint32_t dt)
{
	for (uint32_t t = t0;; t += dt) {
		const uint64_t i = 2ull * s * t;
		if (i >= n)
			break;
		const int32_t c = y[i];
		if (i == 0)
			y[0] = (int16_t)(c - (int16_t)((int32_t)y[s] >> 1));
		else if (i + s < n)
			y[i] = (int16_t)(c - (int16_t)(((int32_t)y[i - s] + (int32_t)y[i + s]) >> 2));
		else
			y[i] = (int16_t)(c - (int16_t)((int32_t)y[i - s] >> 1));
	}
}

template <typename P>
__device__ __forceinline__ void iiwt_odds(P y, uint32_t n, uint32_t s, uint32_t t0, uint32_t dt)
{
	for (uint32_t t = t0;; t += dt) {
		const uint64_t i = (uint64_t)s + 2ull * s * t;
		if (i >= n)
			break;
		const int32_t c = y[i];
		y[i] = i + s < n ? (int16_t)(c + (int16_t)(((int32_t)y[i - s] + (int32_t)y[i + s]) >> 1))
				 : (int16_t)(c + (int32_t)y[i - s]);
	}
}

#define DEC_IWT_LDS_MAX 65536u
// frames up to 64 Ki samples: the whole frame in LDS, one workgroup each
__global__ __launch_bounds__(1024) void dec_iiwt_frame_kernel(DecArgs a)
{
	extern __shared__ int16_t L_f[];
	const uint32_t f = blockIdx.x, t = threadIdx.x;
	const DecInfo I = a.info[f];
	if (I.status || I.pre != 2u || I.n > DEC_IWT_LDS_MAX || I.n < 2u)
		return;
	int16_t *x = reinterpret_cast<int16_t *>(a.dst + (uint64_t)f * (a.dst_stride / 2u));
	for (uint32_t i = t; i < I.n; i += 1024u)
		L_f[i] = x[i];
	__syncthreads();
	uint32_t top = 1;
	while (2u * top < I.n)
		top <<= 1;
	for (uint32_t s = top; s; s >>= 1) {
		iiwt_evens(L_f, I.n, s, t, 1024u);
		__syncthreads();
		iiwt_odds(L_f, I.n, s, t, 1024u);
		__syncthreads();
	}
	for (uint32_t i = t; i < I.n; i += 1024u)
		x[i] = L_f[i];
}

// larger frames: one launch per phase per level, in place in dst
__global__ __launch_bounds__(256) void dec_iiwt_level_kernel(DecArgs a, uint32_t s, uint32_t odds)
{
	const uint32_t f = blockIdx.y;
	const DecInfo I = a.info[f];
	if (I.status || I.pre != 2u || I.n <= DEC_IWT_LDS_MAX || s >= I.n)
		return;
	int16_t *x = reinterpret_cast<int16_t *>(a.dst + (uint64_t)f * (a.dst_stride / 2u));
	const uint32_t t0 = blockIdx.x * 256u + threadIdx.x, dt = gridDim.x * 256u;
	if (odds)
		iiwt_odds(x, I.n, s, t0, dt);
	else
		iiwt_evens(x, I.n, s, t0, dt);
}

// MODEL (preprocess.c:406-411) inverse: x[i] = r[i] + model[i] (int16 wrap)
__global__ __launch_bounds__(256) void dec_model_kernel(DecArgs a)
{
	const uint32_t f = blockIdx.y, t = blockIdx.x * 256u + threadIdx.x;
	const DecInfo I = a.info[f];
	if (I.status || I.pre != 3u)
		return;
	uint16_t *x = a.dst + (uint64_t)f * (a.dst_stride / 2u);
	const uint16_t *m = reinterpret_cast<const uint16_t *>(reinterpret_cast<const uint8_t *>(a.model) +
							       (uint64_t)f * a.model_stride);
	for (uint32_t i = t; i < I.n; i += gridDim.x * 256u)
		x[i] = (uint16_t)(x[i] + m[i]);
}

__global__ void dec_status_kernel(DecArgs a)
{
	const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
	if (f >= a.num_frames)
		return;
	const DecInfo I = a.info[f];
	a.status[f] = I.status ? I.status : I.n;
}

} // namespace airsdec

using namespace airsdec;

#define DCHECK(x)                                   \
	do {                                        \
		if ((x) != hipSuccess)              \
			return ERRV(E_GENERIC);     \
	} while (0)

// Decode num_frames frames (device) into 16-bit samples (device); status[f] =
// samples decoded or an error value.  Synchronises with the host to size the
// parse and to test for a settled parse.
extern "C" uint32_t airs_dev_decode(struct airs_dev_engine *e, const void *src, uint64_t src_stride,
				   uint32_t src_cap, uint32_t num_frames, uint16_t *dst, uint64_t dst_stride,
				   uint32_t dst_samples, uint32_t *status, const uint16_t *model, uint64_t model_stride)
{
	if (!e || !src || !dst || !status || !num_frames || (src_stride & 7u) || ((uintptr_t)src & 7u) ||
	    ((uintptr_t)dst & 1u) || (dst_stride & 1u))
		return ERRV(E_GENERIC);
	hipStream_t s = (hipStream_t)airs_dev_engine_stream(e);
	DecArgs a;
	memset(&a, 0, sizeof(a));
	a.src = (const uint8_t *)src;
	a.src_stride = src_stride;
	a.src_cap = src_cap;
	a.num_frames = num_frames;
	a.dst = dst;
	a.dst_stride = dst_stride;
	a.dst_samples = dst_samples;
	a.status = status;
	a.model = model;
	a.model_stride = model_stride;
	// frame info + the largest subsequence count
	uint8_t *hdr = (uint8_t *)airs_dev_scratch(e, AIRS_NSLOT - 2, (size_t)num_frames * sizeof(DecInfo) + 64u);
	if (!hdr)
		return ERRV(E_GENERIC);
	a.info = (DecInfo *)hdr;
	a.maxsub = (uint32_t *)(hdr + (size_t)num_frames * sizeof(DecInfo));
	a.changed = a.maxsub + 1;
	DCHECK(hipMemsetAsync(a.maxsub, 0, 12, s));
	hipLaunchKernelGGL(dec_hdr_kernel, dim3((num_frames + 255u) / 256u), dim3(256), 0, s, a);
	uint32_t hv[3] = {0, 0, 0}; // largest subsequence count, (changed), any IWT frame
	DCHECK(hipMemcpyAsync(hv, a.maxsub, 12, hipMemcpyDeviceToHost, s));
	DCHECK(hipStreamSynchronize(s));
	const uint32_t msub = hv[0];
	const bool any_iwt = hv[2] != 0u;
	a.msub = msub ? msub : 1u;
	const uint32_t max_n = dst_samples;
	const uint32_t tiles = (max_n + DEC_TILE - 1u) / DEC_TILE;
	a.mwg = (a.msub + DEC_WG - 1u) / DEC_WG;
	const size_t per = (size_t)num_frames * a.msub * 4u, per_wg = (size_t)num_frames * a.mwg * 4u;
	const size_t need = 4u * per + 2u * per_wg + (size_t)num_frames * tiles * 2u + 64u;
	// the decoder's own slot (the device layer keeps AIRS_NSLOT-1 for IWT)
	uint8_t *big = (uint8_t *)airs_dev_scratch(e, AIRS_NSLOT - 3, need);
	if (!big)
		return ERRV(E_GENERIC);
	a.exit_a = (uint32_t *)big;
	a.exit_b = (uint32_t *)(big + per);
	a.cnt = (uint32_t *)(big + 2u * per);
	a.base = (uint32_t *)(big + 3u * per);
	a.wg_cnt = (uint32_t *)(big + 4u * per);
	a.wg_base = (uint32_t *)(big + 4u * per + per_wg);
	a.tile_sum = (uint16_t *)(big + 4u * per + 2u * per_wg);
	if (msub) {
		const dim3 grid(a.mwg, num_frames);
		if (num_frames > 65535u)
			return ERRV(E_GENERIC);
		uint32_t *ein = a.exit_a, *eout = a.exit_b;
		hipLaunchKernelGGL(dec_parse_kernel, grid, dim3(DEC_WG), 0, s, a, (const uint32_t *)nullptr, ein, 1u);
		// rounds until no workgroup's last exit moves (each round passes the
		// corrections one workgroup on, so mwg + 1 rounds always settle)
		for (uint32_t round = 1; round <= a.mwg + 1u; round++) {
			DCHECK(hipMemsetAsync(a.changed, 0, 4, s));
			hipLaunchKernelGGL(dec_parse_kernel, grid, dim3(DEC_WG), 0, s, a, (const uint32_t *)ein, eout, 0u);
			uint32_t *tmp = ein;
			ein = eout;
			eout = tmp;
			uint32_t ch = 1;
			DCHECK(hipMemcpyAsync(&ch, a.changed, 4, hipMemcpyDeviceToHost, s));
			DCHECK(hipStreamSynchronize(s));
			if (!ch)
				break;
		}
		hipLaunchKernelGGL(dec_scan_kernel, dim3(num_frames), dim3(1024), 0, s, a);
		hipLaunchKernelGGL(dec_out_kernel, grid, dim3(DEC_WG), 0, s, a, (const uint32_t *)ein);
		const dim3 tg(tiles, num_frames);
		hipLaunchKernelGGL(dec_tile_sum_kernel, tg, dim3(256), 0, s, a, tiles);
		hipLaunchKernelGGL(dec_tile_prefix_kernel, dim3(num_frames), dim3(1024), 0, s, a, tiles);
		hipLaunchKernelGGL(dec_tile_scan_kernel, tg, dim3(256), 0, s, a, tiles);
		if (model)
			hipLaunchKernelGGL(dec_model_kernel, dim3(min((max_n + 255u) / 256u, 256u), num_frames), dim3(256), 0,
					   s, a);
		// IWT frames
		static bool attr = false;
		if (!attr) {
			DCHECK(hipFuncSetAttribute((const void *)dec_iiwt_frame_kernel,
						   hipFuncAttributeMaxDynamicSharedMemorySize, (int)(DEC_IWT_LDS_MAX * 2u)));
			attr = true;
		}
		if (any_iwt)
			hipLaunchKernelGGL(dec_iiwt_frame_kernel, dim3(num_frames), dim3(1024),
					   (size_t)min(max_n, DEC_IWT_LDS_MAX) * 2u, s, a);
		if (any_iwt && max_n > DEC_IWT_LDS_MAX) {
			uint32_t top = 1;
			while (2u * top < max_n)
				top <<= 1;
			for (uint32_t st = top; st; st >>= 1) {
				const uint32_t items = (uint32_t)(((uint64_t)max_n + 2ull * st - 1ull) / (2ull * st));
				const dim3 lg(min((items + 255u) / 256u, 1024u), num_frames);
				hipLaunchKernelGGL(dec_iiwt_level_kernel, lg, dim3(256), 0, s, a, st, 0u);
				hipLaunchKernelGGL(dec_iiwt_level_kernel, lg, dim3(256), 0, s, a, st, 1u);
			}
		}
	}
	hipLaunchKernelGGL(dec_status_kernel, dim3((num_frames + 255u) / 256u), dim3(256), 0, s, a);
	DCHECK(hipGetLastError());
	return 0;
}
