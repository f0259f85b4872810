// pbr_build_info.cpp — pbr_hip_build_info(): the content hash of the library's sources (Makefile
// SRC_HASH), which ties PMC summaries and bench lines to a build.  Rebuilt whenever any source changes.
#include "../../include/pbr_hip.h"

#ifndef PBR_SRC_HASH
#define PBR_SRC_HASH "unknown"
#endif
#if defined(PBR_DEV_KNOBS) && PBR_DEV_KNOBS
#define PBR_BUILD_KIND " dev-knobs"   // an A/B build whose tuning switches may differ from the defaults
#else
#define PBR_BUILD_KIND ""
#endif
extern "C" const char* pbr_hip_build_info(void) { return "pbr_hip gfx950 wavefront+megakernel src " PBR_SRC_HASH PBR_BUILD_KIND; }
