/* The oracle (oracle/ik_oracle.c, test infrastructure) under ASan + UBSan: object-graph
 * build, one frame on 1 and on 3 threads (identical bits required), segment table.
 *   oracle_san <case file> */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/mbik_oracle.h"
#include "case_io.h"

int main(int argc, char **argv) {
	if (argc < 2) return 2;
	san_case c = san_load(argv[1]);
	oracle_desc d = {c.B, c.parents, c.P, c.pin_bone, c.pin_weight, c.pin_prio, c.pin_prop, c.C, c.cons_bone,
					 c.cons_ncones, c.max_cones, c.iterations, c.default_damp, c.constraint_mode, c.stab,
					 c.bone_damp_count, c.bone_damp_count ? c.bone_damp : NULL};
	void *h = oracle_create(&d, c.N, c.pose, c.cones, c.twist);
	if (!h) {
		printf("oracle_create refused\n");
		san_free(&c);
		return 0;
	}
	const size_t pose_n = (size_t)c.N * c.B * 10;
	float *a = (float *)malloc(pose_n * 4 + 4), *b = (float *)malloc(pose_n * 4 + 4);
	int rc = oracle_solve(h, 0, c.N, c.pose, c.targets, a, NULL, 1);
	oracle_destroy(h);
	h = oracle_create(&d, c.N, c.pose, c.cones, c.twist);
	rc |= oracle_solve(h, 0, c.N, c.pose, c.targets, b, NULL, 3);
	int32_t root[4096], tip[4096], nh[4096];
	const int ns = oracle_segment_table(h, root, tip, nh, 4096);
	oracle_destroy(h);
	const int same = memcmp(a, b, pose_n * 4) == 0;
	printf("ok rc=%d segments=%d threads_agree=%d\n", rc, ns, same);
	free(a);
	free(b);
	san_free(&c);
	return (rc == 0 && same) ? 0 : 1;
}
