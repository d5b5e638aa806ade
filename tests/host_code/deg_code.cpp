// gc_deg_code (csrc/gc_internal.h) on the CPU: the rank partition's first gather compares
// these byte codes, so the code must be monotone in the degree, exact below
// GC_DEG_CODE_EXACT (equal codes there mean equal degrees) and within a byte.  Checks every
// degree up to 2^20 and a stride of the rest up to 2^31 - 1; prints "ok".
#include <cstdio>

#include "gc_internal.h"

int main() {
    unsigned prev = 0;
    long long checked = 0;
    for (long long d = 0; d < (1ll << 31); d += (d < (1ll << 20) ? 1 : 4099), ++checked) {
        const unsigned c = gc_deg_code(d);
        if (c < prev || c > 255u || (d < (long long)GC_DEG_CODE_EXACT && c != (unsigned)d) ||
            (d >= (long long)GC_DEG_CODE_EXACT && c < GC_DEG_CODE_EXACT)) {
            printf("bad: d=%lld code=%u previous=%u\n", d, c, prev);
            return 1;
        }
        prev = c;
    }
    if (gc_deg_code((1ll << 31) - 1) > 254u || gc_deg_code(-5) != 0u) {
        printf("bad range\n");
        return 1;
    }
    printf("ok %lld\n", checked);
    return 0;
}
