// decode.hip -- MI355X (gfx950) decoder for AIRSPACE frames (SURVEY.md 8(f)
// row 1).  The reference has no decoder ("Decompression not implemented yet",
// programs/airspacecli.c:421-423); the format it inverts is the encoder's:
// header (lib/common/header.c:24-67), Golomb codewords (encoder.c:303-378),
// ZigZag (encoder.c:274-286) and the NONE / DIFF predictors
// (preprocess.c:250-290).  The CPU counterpart used as the test oracle is
// orc_decode (oracle/cmp_oracle.c).
//
// A Golomb stream has no index, so the payload of each frame is cut into
// subsequences of DEC_B bits and parsed in parallel by self-synchronisation:
//   parse 0   thread s decodes codewords from bit s*DEC_B (a guess) until it
//             passes (s+1)*DEC_B and records where it stopped (its exit)
//   parse j   thread s decodes from the exit of thread s-1 of parse j-1;
//             repeated until no exit changes (a wrong guess usually falls
//             into step with the true parse after a few codewords, so one or
//             two rounds settle most frames)
//   scan      per frame, exclusive sum of the symbol counts -> output index
//   output    each thread decodes its settled range again and writes the
//             residuals; DIFF frames then take an inclusive int16 prefix sum.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "airs_dev.h"

namespace airsdec {

#define DEC_B 2048u           // bits per subsequence
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
	uint32_t *exit_a, *exit_b, *cnt, *base, *changed;
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

// 64 stream bits from absolute frame bit position abit (MSB first); words
// past the frame's last are clamped to it (their bits are never used)
__device__ __forceinline__ uint64_t win64(const uint32_t *f32, uint32_t wmax, uint32_t abit)
{
	const uint32_t w = abit >> 5, o = abit & 31u;
	const uint32_t d0 = bswap32(f32[min(w, wmax)]), d1 = bswap32(f32[min(w + 1u, wmax)]),
		       d2 = bswap32(f32[min(w + 2u, wmax)]);
	const uint64_t hi = ((uint64_t)d0 << 32) | d1;
	return o ? (hi << o) | (d2 >> (32u - o)) : hi;
}

// one codeword at the top of the 64-bit window W: returns its length (0 =
// invalid) and m, the mapped value (UNCOMPRESSED: the raw 16 bits)
__device__ __forceinline__ uint32_t dec_window(const DecInfo &I, uint64_t W, uint32_t &m)
{
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

__device__ __forceinline__ uint32_t dec_symbol(const DecInfo &I, const uint32_t *f32, uint32_t p, uint32_t &m)
{
	return dec_window(I, win64(f32, I.wmax, I.hdr_bits + p), m);
}

// Sequential bit reader: the next stream bits MSB-aligned in buf (nv valid,
// zeros below), refilled a dword at a time, so a codeword costs a load only
// every few symbols.  A codeword that does not fit the valid bits (its
// decoded length exceeds nv: any bit it used past them was a fill zero) is
// decoded again from memory.
struct BitReader {
	const uint32_t *f32;
	uint32_t wmax, w, nv, p; // next dword, valid bits, payload bit position
	uint64_t buf;
	__device__ __forceinline__ void init(const DecInfo &I, const uint32_t *f, uint32_t pos)
	{
		f32 = f;
		wmax = I.wmax;
		p = pos;
		const uint32_t abit = I.hdr_bits + pos, w0 = abit >> 5, o = abit & 31u;
		const uint64_t hi = ((uint64_t)bswap32(f32[min(w0, wmax)]) << 32) | bswap32(f32[min(w0 + 1u, wmax)]);
		buf = hi << o;
		nv = 64u - o;
		w = w0 + 2u;
	}
	__device__ __forceinline__ uint32_t next(const DecInfo &I, uint32_t &m)
	{
		if (nv <= 32u) {
			buf |= (uint64_t)bswap32(f32[min(w, wmax)]) << (32u - nv);
			w++;
			nv += 32u;
		}
		uint32_t len = dec_window(I, buf, m);
		if (len > nv || !len) {
			len = dec_symbol(I, f32, p, m); // slow path: straight from memory
			if (!len)
				return 0u;
			init(I, f32, p + len);
			return len;
		}
		buf = len < 64u ? buf << len : 0u;
		nv -= len;
		p += len;
		return len;
	}
};

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

// one parse round; first = the speculative round (starts at s * DEC_B)
__global__ __launch_bounds__(256) void dec_parse_kernel(DecArgs a, const uint32_t *exit_in, uint32_t *exit_out,
							uint32_t first)
{
	const uint32_t f = blockIdx.y, s = blockIdx.x * 256u + threadIdx.x;
	const DecInfo I = a.info[f];
	if (s >= I.nsub)
		return;
	const size_t o = (size_t)f * a.msub + s;
	const uint32_t start = s == 0u ? 0u : first ? s * DEC_B : exit_in[o - 1u];
	if (!first && a.base[o] == start) {
		// same start as last round: same result
		exit_out[o] = exit_in[o];
		return;
	}
	a.base[o] = start; // the start this round used (before the scan reuses the array)
	uint32_t p = start, c = 0;
	if (start != DEC_BAD) {
		const uint32_t *f32 = reinterpret_cast<const uint32_t *>(a.src + (uint64_t)f * a.src_stride);
		const uint32_t end = min((s + 1u) * DEC_B, I.nbits);
		BitReader br;
		br.init(I, f32, start);
		while (p < end) {
			uint32_t m;
			const uint32_t len = br.next(I, m);
			if (!len) {
				p = DEC_BAD;
				break;
			}
			p += len;
			c++;
		}
	}
	exit_out[o] = p;
	a.cnt[o] = c;
	if (!first && p != exit_in[o])
		*a.changed = 1u;
}

// per frame: exclusive scan of the symbol counts (one workgroup)
__global__ __launch_bounds__(1024) void dec_scan_kernel(DecArgs a)
{
	__shared__ uint32_t s_w[16];
	__shared__ uint32_t s_carry;
	const uint32_t f = blockIdx.x, t = threadIdx.x, lane = t & 63u, wid = t >> 6;
	const DecInfo I = a.info[f];
	if (t == 0)
		s_carry = 0;
	__syncthreads();
	for (uint32_t b0 = 0; b0 < I.nsub; b0 += 1024u) {
		const uint32_t s = b0 + t;
		const size_t o = (size_t)f * a.msub + s;
		const uint32_t v = s < I.nsub ? a.cnt[o] : 0u;
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
		if (s < I.nsub)
			a.base[o] = woff + inc - v;
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
__global__ __launch_bounds__(256) void dec_out_kernel(DecArgs a, const uint32_t *exits)
{
	const uint32_t f = blockIdx.y, s = blockIdx.x * 256u + threadIdx.x;
	const DecInfo I = a.info[f];
	if (s >= I.nsub || I.status)
		return;
	const size_t o = (size_t)f * a.msub + s;
	const uint32_t b0 = a.base[o];
	uint32_t p = s ? exits[o - 1u] : 0u, j = b0;
	const uint32_t end = min((s + 1u) * DEC_B, I.nbits);
	const uint32_t *f32 = reinterpret_cast<const uint32_t *>(a.src + (uint64_t)f * a.src_stride);
	uint16_t *out = a.dst + (uint64_t)f * (a.dst_stride / 2u);
	// samples are shifted into a 128-bit register and leave as 16-byte stores
	// of 8 (their run is contiguous; each lane's run starts anywhere), with
	// 2-byte stores for the unaligned ends
	const bool vec = (((uintptr_t)out | a.dst_stride) & 15u) == 0;
	uint64_t lo = 0, hi = 0;
	BitReader br;
	if (p < end)
		br.init(I, f32, p);
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
	const size_t per = (size_t)num_frames * a.msub * 4u;
	const size_t need = 4u * per + (size_t)num_frames * tiles * 2u + 64u;
	// the decoder's own slot (the device layer keeps AIRS_NSLOT-1 for IWT)
	uint8_t *big = (uint8_t *)airs_dev_scratch(e, AIRS_NSLOT - 3, need);
	if (!big)
		return ERRV(E_GENERIC);
	a.exit_a = (uint32_t *)big;
	a.exit_b = (uint32_t *)(big + per);
	a.cnt = (uint32_t *)(big + 2u * per);
	a.base = (uint32_t *)(big + 3u * per);
	a.tile_sum = (uint16_t *)(big + 4u * per);
	if (msub) {
		const dim3 grid((a.msub + 255u) / 256u, num_frames);
		if (num_frames > 65535u)
			return ERRV(E_GENERIC);
		uint32_t *ein = a.exit_a, *eout = a.exit_b;
		hipLaunchKernelGGL(dec_parse_kernel, grid, dim3(256), 0, s, a, (const uint32_t *)nullptr, ein, 1u);
		// rounds until no exit moves (two before the first test)
		for (uint32_t round = 1; round <= a.msub + 1u; round++) {
			DCHECK(hipMemsetAsync(a.changed, 0, 4, s));
			hipLaunchKernelGGL(dec_parse_kernel, grid, dim3(256), 0, s, a, (const uint32_t *)ein, eout, 0u);
			uint32_t *tmp = ein;
			ein = eout;
			eout = tmp;
			if (round >= 2u) {
				uint32_t ch = 1;
				DCHECK(hipMemcpyAsync(&ch, a.changed, 4, hipMemcpyDeviceToHost, s));
				DCHECK(hipStreamSynchronize(s));
				if (!ch)
					break;
			}
		}
		hipLaunchKernelGGL(dec_scan_kernel, dim3(num_frames), dim3(1024), 0, s, a);
		hipLaunchKernelGGL(dec_out_kernel, grid, dim3(256), 0, s, a, (const uint32_t *)ein);
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
