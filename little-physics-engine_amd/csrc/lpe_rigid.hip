// lpe_rigid.hip — rigid-body path (placeholder until the rigid kernels land).
#include "lpe_internal.h"
int lpe_rigid_destroy_internal(lpe_ctx *ctx) { (void)ctx; return LPE_OK; }
