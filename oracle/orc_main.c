/*
 * oracle/orc_main.c -- TEST INFRASTRUCTURE ONLY (see orc.h header).
 * `orc <regions|strand_shift|tags_in_regions> [reference CLI flags...]`
 * runs the CPU restatement of the corresponding reference binary.
 */
#include "orc.h"

#include <stdio.h>
#include <string.h>

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: orc regions|strand_shift|tags_in_regions ...\n");
        return 2;
    }
    if (strcmp(argv[1], "regions") == 0) return orc_regions_main(argc - 1, argv + 1);
    if (strcmp(argv[1], "strand_shift") == 0) return orc_strand_shift_main(argc - 1, argv + 1);
    if (strcmp(argv[1], "tags_in_regions") == 0) return orc_tags_in_regions_main(argc - 1, argv + 1);
    fprintf(stderr, "unknown tool %s\n", argv[1]);
    return 2;
}
