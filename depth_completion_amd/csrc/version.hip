// ABI version of libdcamd.so (bumped whenever include/dcamd.h changes incompatibly).
#include "common.h"
#include "../../include/dcamd.h"
extern "C" int dc_abi_version(void) { return 12; }
