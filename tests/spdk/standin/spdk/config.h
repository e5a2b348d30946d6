/* Stand-in for the reference's generated include/spdk/config.h (written by its
 * ./configure, which is not run here).  raid5_simple.c:3 includes it and uses
 * none of its SPDK_CONFIG_* macros, so it defines nothing.  Used ONLY by the
 * tests/spdk harness builds. */
#ifndef SPDK_CONFIG_H
#define SPDK_CONFIG_H
#endif
