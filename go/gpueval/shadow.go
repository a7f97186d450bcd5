package gpueval

// Shadow mode (SURVEY.md 8(b)): one GPU score plugin per replaced reference score plugin.  Each
// returns that plugin's device-computed, already normalized 0-100 value for the node (the cycle
// record GpuEval.PreFilter wrote, kgpu_get_scores), so the profile can keep the reference weights on
// the shadow plugins and the framework applies them exactly as it does to the in-tree plugins:
// range check [0, MaxNodeScore], weight, sum (framework.go:632-648; generic_scheduler.go:660-668),
// then the reference selectHost.
//
// Registration (INTEGRATION.md section 3): for every replaced score plugin,
//   app.WithPlugin(gpueval.ShadowName("NodeResourcesLeastAllocated"), gpueval.NewShadow("NodeResourcesLeastAllocated"))
// or all of them at once through ShadowPlugins().  The profile enables GpuEval at preFilter / filter
// (mode "shadow" in its args) and the shadow plugins at score with the reference weights.

import (
	"context"
	"fmt"

	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/runtime"
	framework "k8s.io/kubernetes/pkg/scheduler/framework/v1alpha1"
)

// ShadowName is the registered name of the shadow plugin of a reference score plugin.
func ShadowName(ref string) string { return "Gpu" + ref }

// GpuScore is the shadow of one reference score plugin.
type GpuScore struct {
	ref string
	id  int32
}

func (s *GpuScore) Name() string { return ShadowName(s.ref) }

// Score returns the device-normalized value of the replaced plugin for the node.  No NormalizeScore:
// DefaultNormalizeScore / the plugins' own normalizations ran on the device over the feasible set.
func (s *GpuScore) Score(ctx context.Context, cs *framework.CycleState, pod *v1.Pod, node string) (int64, *framework.Status) {
	c, err := readCycle(cs)
	if err != nil {
		return 0, framework.NewStatus(framework.Error, err.Error())
	}
	norm, ok := c.norm[s.id]
	if !ok {
		return 0, framework.NewStatus(framework.Error,
			fmt.Sprintf("%s: GpuEval did not run %s (shadow mode, with the plugin in its args)", s.Name(), s.ref))
	}
	i, ok := c.index[node]
	if !ok || int(i) >= len(norm) {
		return 0, framework.NewStatus(framework.Error, fmt.Sprintf("node %q is not in the device mirror", node))
	}
	return norm[i], nil
}

func (s *GpuScore) ScoreExtensions() framework.ScoreExtensions { return nil }

// NewShadow is the framework.PluginFactory (registry.go:28) of the shadow of `ref`.
func NewShadow(ref string) framework.PluginFactory {
	return func(obj runtime.Object, h framework.FrameworkHandle) (framework.Plugin, error) {
		id, ok := scoreIDs[ref]
		if !ok {
			return nil, fmt.Errorf("gpueval: %q is not a score plugin the device implements", ref)
		}
		return &GpuScore{ref: ref, id: id}, nil
	}
}

// ShadowPlugins: the shadow plugin factories of every score plugin the device implements, by
// registered name.
func ShadowPlugins() map[string]framework.PluginFactory {
	out := make(map[string]framework.PluginFactory, len(scoreIDs))
	for ref := range scoreIDs {
		out[ShadowName(ref)] = NewShadow(ref)
	}
	return out
}

var _ framework.ScorePlugin = &GpuScore{}
