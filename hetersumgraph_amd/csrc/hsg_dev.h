// hsg_dev.h -- development-only switches.
//
// The product library (python -m hetersumgraph_amd.build) is compiled without
// HSG_DEV: every HSG_DEV_ENV(...) is a null pointer, so each switch folds to the
// measured default and the library carries no environment-driven dispatch.  The
// dev library (HSG_DEV_BUILD=1 -> libhsg_dev.so, loaded through HSG_LIB_PATH)
// defines HSG_DEV: the switches read the environment again and the rejected
// variants are compiled in for the A/B tools under tools/.
#pragma once
#include <stdlib.h>

#ifdef HSG_DEV
#define HSG_DEV_ENV(name) getenv(name)
#else
#define HSG_DEV_ENV(name) ((const char *)nullptr)
#endif
