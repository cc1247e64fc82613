// Error reporting and version for libirads.so (C ABI: include/irads.h).
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace irads {
static thread_local char g_err[512] = "";
void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace irads

extern "C" const char *irads_last_error(void) { return irads::g_err; }
extern "C" int irads_version(void) { return 1; }
