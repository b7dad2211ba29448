/*
 * cmp_gather.c -- the multi-GPU gather of compressed frames for C callers
 * (include/cmp_gpu.h: cmp_gpu_gather_plan, cmp_gpu_gather).  SURVEY.md 8(e);
 * the protocol of airs-compression_amd/shard.py, over
 * an RCCL communicator the caller owns (one process per GPU):
 *
 *   1. all-gather of one 64-bit entry per frame: its compressed size (or
 *      error value) | the identifier draws it made << 32
 *      (cmp_gpu_batch.draws);
 *   2. every rank packs its frames back to back at 8-byte aligned offsets
 *      (cmp_gpu_pack_frames: reads only the compressed bytes);
 *   3. the root receives every peer's packed bytes straight into its slice of
 *      the output, one group of point-to-point transfers (RCCL has no gatherv;
 *      a group maps onto the direct xGMI link between each pair);
 *   4. the root's frame table in global frame order, and on request the
 *      48-bit header identifiers (bytes 8..13, lib/common/header.c:60-62)
 *      that ONE process would have drawn for the node's frames in global
 *      order with the reference's default counter (lib/compress/cmp.c:27-50):
 *      base + the inclusive scan of the draws.
 *
 * Every rank computes the same plan from the same all-gathered table, so a
 * refusal (a frame with an error value; a frame layout with a frame that made
 * no draw, i.e. a secondary pass that depended on its rank's previous frame;
 * a root capacity below the packed bytes) is decided by all ranks alike,
 * before any point-to-point transfer.  Local failures (arguments, host or
 * device allocations, the packing) go through two small status exchanges, so
 * they too are returned by every rank (cmp_gpu_gather below).
 *
 * RCCL is loaded on first use (dlopen), so the library has no link-time
 * dependency on it.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <rccl/rccl.h>

#include "cmp_errors.h"
#include "cmp_gpu.h"
#include "airs_dev.h"
#include "cmp_engine.h"

#define ERRV(code) ((uint32_t)0u - (uint32_t)CMP_ERR_##code)
#define ID_MASK ((1ull << 48) - 1u)

/* cmp error values are (uint32)-code with code < 128 */
static int size_is_err(uint32_t v)
{
	return v > 0xFFFFFF80u;
}

static uint64_t round8(uint64_t x)
{
	return (x + 7u) & ~(uint64_t)7u;
}

/* global frame number of rank r's local frame j (shard.py global_frame_ids) */
static uint64_t global_frame(uint32_t layout, uint32_t r, uint32_t world, uint32_t fpr, uint32_t fpc, uint32_t j)
{
	switch (layout) {
	case CMP_GPU_LAYOUT_ROUNDROBIN:
		return r + (uint64_t)world * j;
	case CMP_GPU_LAYOUT_STREAMS:
		return ((uint64_t)r + (uint64_t)world * (j / fpc)) * fpc + j % fpc;
	default:
		return (uint64_t)r * fpr + j;
	}
}

uint32_t cmp_gpu_gather_plan(const uint64_t *entries, uint32_t world, uint32_t frames_per_rank, uint32_t layout,
			     uint32_t fpc, uint64_t id_base, uint64_t *rank_bytes, uint64_t *offsets, uint32_t *sizes,
			     uint64_t *ids)
{
	const uint64_t total = (uint64_t)world * frames_per_rank;
	uint64_t base = 0, acc, unit_acc = 0;
	uint32_t r, j;
	uint64_t g;
	uint8_t *dr = NULL;

	if (!entries || !world || !rank_bytes || !offsets || !sizes || layout > CMP_GPU_LAYOUT_STREAMS)
		return ERRV(GENERIC);
	if (layout == CMP_GPU_LAYOUT_STREAMS && (!fpc || frames_per_rank % fpc))
		return ERRV(PARAMS_INVALID);
	/* packed offsets per rank, in global order */
	for (r = 0; r < world; r++) {
		uint64_t off = 0;

		for (j = 0; j < frames_per_rank; j++) {
			const uint32_t sz = (uint32_t)entries[(uint64_t)r * frames_per_rank + j];

			if (size_is_err(sz))
				return ERRV(GENERIC); /* a frame that failed: no size to gather */
			g = global_frame(layout, r, world, frames_per_rank, fpc, j);
			offsets[g] = base + off;
			sizes[g] = sz;
			off += round8(sz);
		}
		rank_bytes[r] = off;
		base += off;
	}
	if (!ids)
		return 0;
	/* identifiers: the draws in global order (shard.py assign_identifiers) */
	dr = malloc(total ? total : 1);
	if (!dr)
		return ERRV(GENERIC);
	for (r = 0; r < world; r++)
		for (j = 0; j < frames_per_rank; j++)
			dr[global_frame(layout, r, world, frames_per_rank, fpc, j)] =
				(uint8_t)(entries[(uint64_t)r * frames_per_rank + j] >> 32);
	acc = id_base;
	for (g = 0; g < total; g++) {
		/* a frame layout is one context over every frame; "streams" one per stream */
		if (layout == CMP_GPU_LAYOUT_STREAMS ? g % fpc == 0 : g == 0)
			unit_acc = 0;
		if (layout != CMP_GPU_LAYOUT_STREAMS && dr[g] == 0) {
			free(dr);
			return ERRV(PARAMS_INVALID); /* a secondary pass: use the streams layout */
		}
		acc += dr[g];
		unit_acc += dr[g];
		/* before its context's first draw a frame keeps the identifier it carries */
		ids[g] = unit_acc ? (acc & ID_MASK) : UINT64_MAX;
	}
	free(dr);
	return 0;
}

/* ---------------- RCCL, loaded on first use ---------------- */
static struct {
	pthread_once_t once;
	int ok;
	ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
	ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
	ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
	ncclResult_t (*group_start)(void);
	ncclResult_t (*group_end)(void);
	ncclResult_t (*count)(const ncclComm_t, int *);
	ncclResult_t (*user_rank)(const ncclComm_t, int *);
	const char *(*err_string)(ncclResult_t);
} R = {PTHREAD_ONCE_INIT, 0, 0, 0, 0, 0, 0, 0, 0, 0};

static void rccl_bind(void *h)
{
	*(void **)&R.all_gather = dlsym(h, "ncclAllGather");
	*(void **)&R.send = dlsym(h, "ncclSend");
	*(void **)&R.recv = dlsym(h, "ncclRecv");
	*(void **)&R.group_start = dlsym(h, "ncclGroupStart");
	*(void **)&R.group_end = dlsym(h, "ncclGroupEnd");
	*(void **)&R.count = dlsym(h, "ncclCommCount");
	*(void **)&R.user_rank = dlsym(h, "ncclCommUserRank");
	*(void **)&R.err_string = dlsym(h, "ncclGetErrorString");
	R.ok = R.all_gather && R.send && R.recv && R.group_start && R.group_end && R.count && R.user_rank &&
	       R.err_string;
}

static void rccl_load(void)
{
	void *h;

	/* the copy the process already holds (the caller made its communicator
	 * with it), else librccl */
	rccl_bind(RTLD_DEFAULT);
	if (R.ok)
		return;
	h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
	if (!h)
		h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
	if (!h) {
		fprintf(stderr, "airscmp: cmp_gpu_gather: RCCL not found (%s)\n", dlerror());
		return;
	}
	rccl_bind(h);
	if (!R.ok)
		fprintf(stderr, "airscmp: cmp_gpu_gather: RCCL lacks a symbol\n");
}

#define NCCL_OK(x)                                                                                   \
	do {                                                                                         \
		ncclResult_t _r = (x);                                                               \
		if (_r != ncclSuccess) {                                                             \
			fprintf(stderr, "airscmp: cmp_gpu_gather: %s: %s\n", #x, R.err_string(_r)); \
			e = ERRV(GENERIC);                                                           \
			goto out;                                                                    \
		}                                                                                    \
	} while (0)

/*
 * One status exchange: every rank contributes {status, value} (status 0 or
 * a cmp error value) through the engine's collective words (allocated with
 * the engine: taking part never needs an allocation), and every rank gets the
 * same answer: the first non-zero status in rank order, or 0.  values[r] is
 * rank r's value.  A rank that failed locally still takes part, so its peers
 * learn of the failure instead of waiting for it in a later collective.
 */
static uint32_t status_exchange(struct airs_dev_engine *dev, ncclComm_t comm, hipStream_t st, int world,
				uint32_t status, uint64_t value, uint64_t *values)
{
	uint64_t rec[2] = {status, value}, all[2 * AIRS_COLL_MAX_RANKS];
	uint64_t *d = airs_dev_coll(dev);
	uint32_t e = 0, first = 0;
	int r;

	/* an upload that fails still leaves the rank in the all-gather */
	if (airs_dev_h2d(dev, d, rec, sizeof(rec)))
		first = ERRV(GENERIC);
	NCCL_OK(R.all_gather(d, d + 2, sizeof(rec), ncclUint8, comm, st));
	e = airs_dev_d2h(dev, all, d + 2, (size_t)world * sizeof(rec));
	if (!e)
		e = airs_dev_sync(dev);
	if (e)
		goto out;
	for (r = 0; r < world; r++) {
		if (!first && (uint32_t)all[2 * r])
			first = (uint32_t)all[2 * r];
		if (values)
			values[r] = all[2 * r + 1];
	}
	e = first;
out:
	return e;
}

/*
 * Every refusal is collective: argument, allocation and packing failures of
 * any rank are folded into a status exchange that every rank enters before
 * the next collective (and the root's out_capacity travels in the first
 * one), so all ranks return the same value and none is left inside an RCCL
 * call.  Only an engine or communicator of NULL, a world over
 * AIRS_COLL_MAX_RANKS, or a missing RCCL returns at once: such a rank cannot
 * take part at all.
 */
uint32_t cmp_gpu_gather(struct cmp_gpu_engine *engine, void *nccl_comm, uint32_t root, uint32_t layout, uint32_t fpc,
			const void *frames, uint64_t frame_stride, uint32_t frame_capacity, const uint32_t *sizes,
			const uint8_t *draws, uint32_t frames_per_rank, void *out, uint64_t out_capacity,
			uint64_t *out_offsets, uint32_t *out_sizes, uint64_t id_base, uint32_t flags)
{
	struct airs_dev_engine *dev;
	ncclComm_t comm = (ncclComm_t)nccl_comm;
	hipStream_t st;
	int rank = 0, world = 0;
	uint32_t e = 0, local = 0, j, r;
	uint64_t *h_loc = NULL, *h_all = NULL, *rank_bytes = NULL, *offs = NULL, *ids = NULL, base = 0, all = 0;
	uint64_t *d_loc = NULL, *d_all = NULL, *d_po = NULL, *d_p = NULL, caps[AIRS_COLL_MAX_RANKS];
	uint32_t *h_sizes = NULL, *fsz = NULL;
	uint8_t *buf = NULL;
	uint64_t total;
	const int patch = (flags & CMP_GPU_GATHER_PATCH_IDS) != 0;

	if (!engine || !nccl_comm)
		return ERRV(GENERIC);
	pthread_once(&R.once, rccl_load);
	if (!R.ok)
		return ERRV(GENERIC);
	dev = engine->dev;
	st = (hipStream_t)airs_dev_engine_stream(dev);
	if (R.count(comm, &world) != ncclSuccess || R.user_rank(comm, &rank) != ncclSuccess || world < 1 ||
	    world > AIRS_COLL_MAX_RANKS)
		return ERRV(GENERIC);
	/* ---- local checks and allocations: their outcome goes into exchange 1 */
	if (root >= (uint32_t)world || !frames || !sizes || !frames_per_rank)
		local = ERRV(GENERIC);
	else if ((uint32_t)rank == root && (!out || !out_offsets || !out_sizes))
		local = ERRV(GENERIC);
	else if ((uint32_t)rank == root && ((uintptr_t)out & 7u))
		local = ERRV(DST_TOO_SMALL);
	total = (uint64_t)world * frames_per_rank;
	if (!local) {
		h_loc = malloc((size_t)frames_per_rank * 8u);
		h_sizes = malloc((size_t)frames_per_rank * 4u);
		h_all = malloc((size_t)total * 8u);
		rank_bytes = malloc((size_t)world * 8u);
		offs = malloc((size_t)total * 8u);
		fsz = malloc((size_t)total * 4u);
		ids = patch ? malloc((size_t)total * 8u) : NULL;
		d_loc = airs_dev_scratch(dev, AIRS_SLOT_GATHER, (size_t)(frames_per_rank + total) * 8u);
		if (!h_loc || !h_sizes || !h_all || !rank_bytes || !offs || !fsz || (patch && !ids) || !d_loc)
			local = ERRV(GENERIC);
	}
	if (!local) {
		/* this rank's table entries: size | draws << 32 (one read-back) */
		local = airs_dev_d2h(dev, h_sizes, sizes, (size_t)frames_per_rank * 4u);
		if (!local)
			local = airs_dev_sync(dev);
		for (j = 0; !local && j < frames_per_rank; j++)
			h_loc[j] = (uint64_t)h_sizes[j] | ((uint64_t)(draws ? draws[j] : 1u) << 32);
	}
	/* ---- exchange 1: every rank's status, the root's capacity */
	e = status_exchange(dev, comm, st, world, local, (uint32_t)rank == root ? out_capacity : 0u, caps);
	if (e)
		goto out;
	/* ---- 1. the size table: the all-gather (d_loc exists on every rank now) */
	d_all = d_loc + frames_per_rank;
	e = airs_dev_h2d(dev, d_loc, h_loc, (size_t)frames_per_rank * 8u);
	if (e)
		goto out;
	NCCL_OK(R.all_gather(d_loc, d_all, (size_t)frames_per_rank * 8u, ncclUint8, comm, st));
	e = airs_dev_d2h(dev, h_all, d_all, (size_t)total * 8u);
	if (!e)
		e = airs_dev_sync(dev);
	if (e)
		goto out;
	/* the same plan on every rank: a refusal is decided before any transfer */
	e = cmp_gpu_gather_plan(h_all, (uint32_t)world, frames_per_rank, layout, fpc, id_base, rank_bytes, offs, fsz,
				ids);
	if (e)
		goto out;
	for (r = 0; r < (uint32_t)world; r++)
		all += rank_bytes[r];
	if (caps[root] < all) {
		e = ERRV(DST_TOO_SMALL); /* decided from the table: on every rank */
		goto out;
	}
	for (j = 0; j < (uint32_t)rank; j++)
		base += rank_bytes[j];
	/* ---- 2. pack (the root into its slice of out, the others into scratch) */
	{
		const uint64_t mine = rank_bytes[rank];

		local = 0;
		d_po = airs_dev_scratch(dev, AIRS_SLOT_GATHER + 1, (size_t)(frames_per_rank + 1) * 8u +
									 ((uint32_t)rank == root ? 0u : mine));
		/* the root's identifier table too: after the transfers nothing is
		 * allocated, so nothing can fail on the root alone */
		if ((uint32_t)rank == root && patch)
			d_p = airs_dev_scratch(dev, AIRS_SLOT_GATHER + 2, (size_t)total * 16u);
		if (!d_po || ((uint32_t)rank == root && patch && !d_p))
			local = ERRV(GENERIC);
		else {
			buf = (uint32_t)rank == root ? (uint8_t *)out + base : (uint8_t *)(d_po + frames_per_rank + 1);
			local = cmp_gpu_pack_frames(engine, frames, frame_stride, frame_capacity, sizes, frames_per_rank,
						    buf, d_po);
			if (!local)
				local = airs_dev_sync(dev);
		}
		/* ---- exchange 2: every rank packed, or none sends */
		e = status_exchange(dev, comm, st, world, local, 0u, NULL);
		if (e)
			goto out;
		/* ---- 3. one group of point-to-point transfers to the root */
		NCCL_OK(R.group_start());
		if ((uint32_t)rank == root) {
			uint64_t b = 0;

			for (r = 0; r < (uint32_t)world; r++) {
				if (r != root && rank_bytes[r]) {
					ncclResult_t q = R.recv((uint8_t *)out + b, rank_bytes[r], ncclUint8, (int)r, comm, st);

					if (q != ncclSuccess) {
						(void)R.group_end();
						NCCL_OK(q);
					}
				}
				b += rank_bytes[r];
			}
		} else if (mine) {
			ncclResult_t q = R.send(buf, mine, ncclUint8, (int)root, comm, st);

			if (q != ncclSuccess) {
				(void)R.group_end();
				NCCL_OK(q);
			}
		}
		NCCL_OK(R.group_end());
	}
	if ((uint32_t)rank != root) {
		e = airs_dev_sync(dev); /* the send has left this rank's scratch */
		goto out;
	}
	/* ---- 4. the root: frame table in global order, identifiers into the headers */
	memcpy(out_offsets, offs, (size_t)total * 8u);
	memcpy(out_sizes, fsz, (size_t)total * 4u);
	if (patch) {
		uint64_t n = 0, g;

		for (g = 0; g < total; g++)
			if (ids[g] != UINT64_MAX && fsz[g] >= 14u) {
				offs[n] = offs[g];
				ids[n] = ids[g];
				n++;
			}
		if (n) {
			e = airs_dev_h2d(dev, d_p, offs, (size_t)n * 8u);
			if (!e)
				e = airs_dev_h2d(dev, d_p + n, ids, (size_t)n * 8u);
			if (!e)
				e = airs_dev_patch_ids_at(dev, out, d_p, d_p + n, n);
		}
	}
	if (!e)
		e = airs_dev_sync(dev); /* the host arrays below are freed next */
out:
	free(h_loc);
	free(h_sizes);
	free(h_all);
	free(rank_bytes);
	free(offs);
	free(fsz);
	free(ids);
	return e;
}
