// Host build of ngrtd_fastmath.hpp for tests/test_fastmath_cpu.py:
//   reads "e x" / "l x" lines (hex doubles) from stdin, prints results as hex doubles.
#include "../noblegas_rtd_mcmc_amd/csrc/ngrtd_fastmath.hpp"
#include <cstdio>
#include <cstdlib>
#include <cstring>
int main() {
    char op;
    unsigned long long bits;
    while (scanf(" %c %llx", &op, &bits) == 2) {
        double x;
        memcpy(&x, &bits, 8);
        double r = (op == 'e') ? ngrtd::fexp(x) : ngrtd::flog(x);
        unsigned long long rb;
        memcpy(&rb, &r, 8);
        printf("%llx\n", rb);
    }
    return 0;
}
