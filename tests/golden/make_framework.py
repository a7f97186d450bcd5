"""Golden vectors transcribed from pkg/scheduler/framework/v1alpha1/framework_test.go: the runner
tables TestRunScorePlugins (:614) and TestFilterPlugins (:838).

Both drive the framework's own loops with test plugins whose outcome is injected (TestPlugin,
TestScorePlugin, TestScoreWithNormalizePlugin; restated in tests/fake_plugins.py):
  * run_score: RunScorePlugins over nodes node1 / node2 -- per-plugin scores after NormalizeScore and
    the weight (defaultWeights: score-with-normalize-plugin-2 has weight 2), or an error when Score or
    NormalizeScore fails or a normalized score leaves [MinNodeScore, MaxNodeScore];
  * run_filter: RunFilterPlugins + PluginToStatus.Merge on one node -- the status map (first failure
    only unless runAllFilters; a non-Unschedulable code becomes an Error naming the plugin) and the
    merged status (precedence Error > UnschedulableAndUnresolvable > Unschedulable)."""
from gen_common import case

SRC = "pkg/scheduler/framework/v1alpha1/framework_test.go"
SUCCESS, ERROR, UNSCHED, UNRES = 0, 1, 2, 3
S1, SN1, SN2 = "score-plugin-1", "score-with-normalize-plugin-1", "score-with-normalize-plugin-2"
WEIGHTS = {SN1: 1, SN2: 2, S1: 1}   # framework_test.go:327-331 defaultWeights
INJ = "injected filter status"


def run_score_cases():
    out = []

    def rs(name, line, plugins, args, want=None, err=False):
        spec = {p: dict(args.get(p, {}), normalize=p != S1) for p in plugins}
        kw = {"expect_error": ""} if err else {"expect_run_scores": {p: [["node1", s], ["node2", s]]
                                                                      for p, s in want.items()}}
        out.append(case(name, SRC + ":%d" % line, kind="run_score",
                        profile={"filters": [], "prefilters": [], "prescores": [],
                                 "scores": [[p, WEIGHTS[p]] for p in plugins], "fake": {"injected_scores": spec}},
                        **kw))

    rs("no Score plugins", 625, [], {}, {})
    rs("single Score plugin", 630, [S1], {S1: {"scoreRes": 1}}, {S1: 1})
    rs("single ScoreWithNormalize plugin", 646, [SN1], {SN1: {"scoreRes": 10, "normalizeRes": 5}}, {SN1: 5})
    rs("2 Score plugins, 2 NormalizeScore plugins", 663, [S1, SN1, SN2],
       {S1: {"scoreRes": 1}, SN1: {"scoreRes": 3, "normalizeRes": 4}, SN2: {"scoreRes": 4, "normalizeRes": 5}},
       {S1: 1, SN1: 4, SN2: 10})
    rs("score fails", 695, [S1, SN1], {SN1: {"scoreStatus": 1}}, err=True)
    rs("normalize fails", 708, [S1, SN1], {SN1: {"normalizeStatus": 1}}, err=True)
    rs("Score plugin return score greater than MaxNodeScore", 721, [S1], {S1: {"scoreRes": 101}}, err=True)
    rs("Score plugin return score less than MinNodeScore", 734, [S1], {S1: {"scoreRes": -1}}, err=True)
    rs("ScoreWithNormalize plugin return score greater than MaxNodeScore", 747, [SN1], {SN1: {"normalizeRes": 101}},
       err=True)
    rs("ScoreWithNormalize plugin return score less than MinNodeScore", 760, [SN1], {SN1: {"normalizeRes": -1}},
       err=True)
    return out


def run_filter_cases():
    out = []

    def rf(name, line, plugins, want_code, want_map, run_all=False, want_reasons=None):
        """plugins: [(name, injected code)]; want_map: {plugin: (code, message)}."""
        err_msg = lambda p: 'running "%s" filter plugin for pod "": %s' % (p, INJ)  # noqa: E731
        wm = {}
        for p, code in want_map.items():
            wm[p] = {"code": code, "reasons": [err_msg(p) if code == ERROR else INJ]}
        merged = None
        if want_code is not None:
            merged = {"code": want_code, "reasons": want_reasons if want_reasons is not None else
                      [r for p in want_map for r in wm[p]["reasons"]]}
        out.append(case(name, SRC + ":%d" % line, kind="run_filter", run_all_filters=run_all,
                        profile={"filters": [p for p, _ in plugins], "prefilters": [], "prescores": [], "scores": [],
                                 "fake": {"injected_filters": {p: c for p, c in plugins}}},
                        expect_status_map=wm, expect_merged=merged))

    T, T1, T2 = "TestPlugin", "TestPlugin1", "TestPlugin2"
    rf("SuccessFilter", 847, [(T, SUCCESS)], None, {})
    rf("ErrorFilter", 858, [(T, ERROR)], ERROR, {T: ERROR})
    rf("UnschedulableFilter", 869, [(T, UNSCHED)], UNSCHED, {T: UNSCHED})
    rf("UnschedulableAndUnresolvableFilter", 880, [(T, UNRES)], UNRES, {T: UNRES})
    rf("ErrorAndErrorFilters", 893, [(T1, ERROR), (T2, ERROR)], ERROR, {T1: ERROR})
    rf("SuccessAndSuccessFilters", 909, [(T1, SUCCESS), (T2, SUCCESS)], None, {})
    rf("ErrorAndSuccessFilters", 925, [(T1, ERROR), (T2, SUCCESS)], ERROR, {T1: ERROR})
    rf("SuccessAndErrorFilters", 940, [(T1, SUCCESS), (T2, ERROR)], ERROR, {T2: ERROR})
    rf("SuccessAndUnschedulableFilters", 956, [(T1, SUCCESS), (T2, UNSCHED)], UNSCHED, {T2: UNSCHED})
    rf("SuccessFilterWithRunAllFilters", 972, [(T, SUCCESS)], None, {}, run_all=True)
    rf("ErrorAndErrorFilters", 984, [(T1, ERROR), (T2, ERROR)], ERROR, {T1: ERROR}, run_all=True)
    rf("ErrorAndErrorFilters", 1001, [(T1, UNRES), (T2, UNSCHED)], UNRES, {T1: UNRES, T2: UNSCHED}, run_all=True,
       want_reasons=[INJ, INJ])
    return out


def all_cases():
    return run_score_cases() + run_filter_cases()
