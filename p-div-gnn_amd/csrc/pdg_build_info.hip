// Build identity of the library: a hash of the sources it was compiled from (csrc/*.hip, csrc/*.hpp,
// include/pdivgnn.h), set by build.py.  pdg.lib refuses a shipped library whose hash differs from
// the sources beside it, so a stale build cannot be measured or tested as the current one.
#include "../../include/pdivgnn.h"

#ifndef PDG_SRC_HASH
#define PDG_SRC_HASH "unknown"
#endif

extern "C" const char* pdg_source_hash(void) { return PDG_SRC_HASH; }
