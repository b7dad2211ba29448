/* cmp_engine.h -- the opaque cmp_gpu_engine of include/cmp_gpu.h (private to
 * the library's host code: cmp_host.c, cmp_gather.c) */
#ifndef CMP_ENGINE_H
#define CMP_ENGINE_H

#include "airs_dev.h"

struct cmp_gpu_engine {
	struct airs_dev_engine *dev;
};

#endif /* CMP_ENGINE_H */
