/* oracle/gamma_exhaustive.c -- TEST INFRASTRUCTURE ONLY (tests/test_gamma_exhaustive.py).
 *
 * Proves hazard H6 away: the reference gammas with glibc powf(x, 0.5f) (renderer.cpp:125-131)
 * and packs with ToBGRA8 (lin_alg.h:125-132); the HIP kernel uses the correctly rounded
 * sqrtf.  For EVERY float x in [0, 0x3F810000] (= [0, 1.0078]; averaged colours lie in
 * [0, 1 + 2 ulp]) this counts inputs where the float results differ and where the packed
 * byte differs.  Above the range both results exceed 1 and pack to 255; negative inputs
 * and NaN give NaN in both, which packs to 0.  Prints "float_diffs N byte_diffs M".
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static unsigned pack(float c)
{
    if (c > 1.0f) return 255u;
    const float x = c * 255.0f;
    int i = (x >= -2147483648.0f && x < 2147483648.0f) ? (int)x : (int)0x80000000u; /* cvttss2si */
    return (unsigned)i & 255u;
}

int main(void)
{
    long nf = 0, nb = 0;
    const long hi = 0x3F810000L;
#pragma omp parallel for reduction(+ : nf, nb) schedule(static)
    for (long b = 0; b <= hi; b++)
    {
        const uint32_t u = (uint32_t)b;
        float x;
        memcpy(&x, &u, 4);
        const float p = powf(x, 0.5f), s = sqrtf(x);
        if (memcmp(&p, &s, 4) != 0)
        {
            nf++;
            if (pack(p) != pack(s)) nb++;
        }
    }
    printf("float_diffs %ld byte_diffs %ld\n", nf, nb);
    return 0;
}
