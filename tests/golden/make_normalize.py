"""Golden vectors transcribed from pkg/scheduler/framework/plugins/helper/normalize_score_test.go."""
from gen_common import case

SRC = "pkg/scheduler/framework/plugins/helper/normalize_score_test.go"
TABLE = [  # (line, reverse, scores, expected)
    (31, False, [1, 2, 3, 4], [25, 50, 75, 100]),
    (35, True, [1, 2, 3, 4], [75, 50, 25, 0]),
    (40, False, [1000, 10, 20, 30], [100, 1, 2, 3]),
    (44, True, [1000, 10, 20, 30], [0, 99, 98, 97]),
    (49, False, [1, 1, 1, 1], [100, 100, 100, 100]),
    (53, False, [1000, 1, 1, 1], [100, 0, 0, 0]),
    (57, True, [0, 1, 1, 1], [100, 0, 0, 0]),
]


def all_cases():
    return [case("DefaultNormalizeScore #%d" % i, SRC + ":%d" % line, kind="normalize", max_priority=100,
                 reverse=rev, scores=[[str(j), s] for j, s in enumerate(sc)],
                 expect_scores={str(j): e for j, e in enumerate(exp)})
            for i, (line, rev, sc, exp) in enumerate(TABLE)]
