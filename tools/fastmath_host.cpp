// Host build of the device math helpers for tests/test_fastmath_cpu.py:
//   reads "<op> x" lines (x as hex double bits) from stdin, prints results as hex bits.
//   op: e = fexp, t = fexp10, l = flog, m = fexpm1, g = lgamma_half_diff (lgamma(x+1/2) - lgamma(x)),
//   p = lapse_rate_fast.
#include "../noblegas_rtd_mcmc_amd/csrc/ngrtd_math.hpp"
#include <cstdio>
#include <cstdlib>
#include <cstring>
int main() {
    char op;
    unsigned long long bits;
    while (scanf(" %c %llx", &op, &bits) == 2) {
        double x;
        memcpy(&x, &bits, 8);
        double r = (op == 'e') ? ngrtd::fexp(x) : (op == 't') ? ngrtd::fexp10(x) : (op == 'l') ? ngrtd::flog(x)
                 : (op == 'm') ? ngrtd::fexpm1(x) : (op == 'p') ? ngrtd::lapse_rate_fast(x) : ngrtd::lgamma_half_diff(x);
        unsigned long long rb;
        memcpy(&rb, &r, 8);
        printf("%llx\n", rb);
    }
    return 0;
}
