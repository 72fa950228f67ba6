/* ORACLE -- test infrastructure only (never linked into the product). */
#ifndef ORACLE_COMMON_H
#define ORACLE_COMMON_H
#include <stdint.h>
#endif
