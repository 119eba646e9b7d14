// zipf_ref_main.cpp — driver that runs the REFERENCE's own zipf generator
// (test/zipf.h of cmemory/Sherman, compiled by path from the reference
// checkout: oracle/Makefile target `ref`, output oracle/_ref/zipf_ref; the
// header is never copied).  It pins the oracle's restatement
// (sherman_oracle.c orc_zipf_*) and tests/golden/generators.json to the
// reference's arithmetic.  Test infrastructure only.
//
// usage: zipf_ref N THETA SEED COUNT   -> COUNT draws, one per line
#include <cstdio>
#include <cstdlib>

#include "zipf.h"  // -I <reference>/test

int main(int argc, char** argv) {
  if (argc != 5) {
    fprintf(stderr, "usage: %s N THETA SEED COUNT\n", argv[0]);
    return 2;
  }
  const uint64_t n = strtoull(argv[1], nullptr, 0);
  const double theta = strtod(argv[2], nullptr);
  const uint64_t seed = strtoull(argv[3], nullptr, 0);
  const long count = strtol(argv[4], nullptr, 0);
  struct zipf_gen_state st;
  mehcached_zipf_init(&st, n, theta, seed);  // test/zipf.h:96-126
  for (long i = 0; i < count; ++i)
    printf("%llu\n", (unsigned long long)mehcached_zipf_next(&st));  // test/zipf.h:163-203
  return 0;
}
