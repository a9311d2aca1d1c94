// ABI version and build id of libdcamd.so.
// dc_abi_version is bumped whenever include/dcamd.h changes incompatibly; dc_build_id is the sha256 prefix of
// the sources the library was compiled from (depth_completion_amd/build.py source_hash), which the loader
// compares with the tree it runs from, so a stale binary is refused even when the ABI number matches.
#include "common.h"
#include "../../include/dcamd.h"
#ifndef DC_BUILD_ID
#define DC_BUILD_ID "unknown"
#endif
extern "C" int dc_abi_version(void) { return 21; }
extern "C" const char* dc_build_id(void) { return DC_BUILD_ID; }
