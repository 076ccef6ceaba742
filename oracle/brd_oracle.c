/*
 * TEST INFRASTRUCTURE ONLY (see brd_oracle_impl.h).  CPU oracle for the
 * two-stage bidiagonal reduction, instantiated for float and double.
 *
 * Build: oracle/Makefile  ->  oracle/liboracle.so
 * Must be compiled WITHOUT fp contraction (-ffp-contract=off) and without
 * -march=native, so that it reproduces the reference fixtures bit for bit.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define OT float
#define OSFX f32
#include "brd_oracle_impl.h"
#undef OT
#undef OSFX

#define OT double
#define OSFX f64
#include "brd_oracle_impl.h"
#undef OT
#undef OSFX

int oracle_abi_version(void) { return 1; }
