/* orc_tauhost: command-line front end of orc_tauhost_main (TEST INFRASTRUCTURE
 * ONLY).  Same 13 positional arguments as the reference's tauhost.c:31-43. */
#include <stdio.h>
#include "sq_oracle.h"
int main(int argc, char **argv) { return orc_tauhost_main(argc, (const char **)argv, stdout); }
