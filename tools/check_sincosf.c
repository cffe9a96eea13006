/* Exhaustive check: the glibc sinf/cosf restatement used by the oracle and by
 * the HIP descriptor kernel equals the host libm on EVERY float in [0, 6.3]
 * (all angles the reference can pass: fastAtan2 degrees * pi/180).
 * Build+run: gcc -O2 -ffp-contract=off tools/check_sincosf.c oracle/liborbref.so -lm && ./a.out */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
float orbref_sinf(float);
float orbref_cosf(float);
int main(void) {
    const float lim = 6.3f;
    uint32_t hi;
    memcpy(&hi, &lim, 4);
    long bad = 0, tot = 0;
    for (uint32_t u = 0; u <= hi; ++u) {
        float f, a, b, c, d;
        memcpy(&f, &u, 4);
        a = sinf(f); b = cosf(f); c = orbref_sinf(f); d = orbref_cosf(f);
        if (memcmp(&a, &c, 4) || memcmp(&b, &d, 4)) { if (bad < 8) printf("mismatch %a\n", f); ++bad; }
        ++tot;
    }
    printf("checked %ld floats, %ld mismatches\n", tot, bad);
    return bad != 0;
}
