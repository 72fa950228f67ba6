/* ORACLE -- placeholder, filled in with the M-step restatement */
#include "oracle_common.h"
int oracle_mstep_version(void) { return 1; }
