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
static thread_local unsigned long long *g_stamp = nullptr;
unsigned long long *take_stamp() {
    unsigned long long *s = g_stamp;
    g_stamp = nullptr;
    return s;
}
}  // namespace irads

extern "C" const char *irads_last_error(void) { return irads::g_err; }
extern "C" void irads_stamp_next(unsigned long long *slot) { irads::g_stamp = slot; }
extern "C" int irads_wall_clock_khz(void) {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess)
        return 0;
    return khz;
}
extern "C" int irads_version(void) { return 1; }
