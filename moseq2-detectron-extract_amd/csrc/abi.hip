// Error state + version of the mdx C ABI.
#include "common.h"

namespace mdx {
static thread_local std::string g_err;
void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}
}  // namespace mdx

extern "C" const char *mdx_last_error(void) { return mdx::g_err.c_str(); }
extern "C" const char *mdx_version(void) { return "mdx 0.1.0 gfx950"; }
