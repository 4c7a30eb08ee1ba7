// errno_guard.hip -- leaves errno as the C runtime started it once the library is loaded.
//
// Each kernel file registers its gfx950 code object from a load-time constructor
// (the HIP module ctor); on the way the runtime probes files that need not exist
// and leaves errno == ENOENT behind.  A program that links libtyche_codec.so
// would then reach main() with errno already set, and the reference trips on
// exactly that: io__scan_for_pages tests errno instead of the DIR* returned by
// opendir (/root/reference/src/io.c:89-93), so tyche would exit at startup with
// "File/directory not found".  C guarantees errno == 0 at program start; this
// constructor restores that.  The build links this object after every kernel
// object (tyche_amd/_build.py SOURCES), and the loader runs a library's
// .init_array in link order, so it runs after all the module constructors.
#include <errno.h>

namespace {
__attribute__((constructor)) void tyche_errno_reset() { errno = 0; }
}  // namespace
