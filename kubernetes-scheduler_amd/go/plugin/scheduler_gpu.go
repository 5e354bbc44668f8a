// Package yoda — GPU-backed variant of the Yoda plugin's extension points
// (pkg/yoda/scheduler.go of Mr-LvGJ/kubernetes-scheduler), served by libyoda through
// yodagpu.  Registration is unchanged: register.go:8-12 keeps
// app.WithPlugin(yoda.Name, yoda.New); New builds a GPU handle instead of the Redis client.
//
// NOT COMPILED HERE (no Go toolchain in the build image); see INTEGRATION.md.
package yoda

import (
	"context"
	"fmt"
	"sync"

	scv "github.com/NJUPT-ISL/SCV/api/v1"
	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/runtime"
	"k8s.io/kubernetes/pkg/scheduler/framework"

	"github.com/Mr-LvGJ/Yoda-Scheduler/pkg/yoda/yodagpu"
)

const Name = "yoda"

var (
	_ framework.PreFilterPlugin = &Yoda{}
	_ framework.FilterPlugin    = &Yoda{}
	_ framework.PreScorePlugin  = &Yoda{}
	_ framework.ScorePlugin     = &Yoda{}
	_ framework.ScoreExtensions = &Yoda{}
	_ framework.PreBindPlugin   = &Yoda{}
	_ framework.QueueSortPlugin = &Yoda{}
)

// SnapshotSource lists the SCV records (core.run-linux.com/scvs, deploy/yoda-scheduler.yaml:
// 225-236) and the allocated scv/memory per node; an informer-backed implementation
// re-uploads the snapshot when it changes.
type SnapshotSource interface {
	Snapshot() (names []string, scvs []*scv.Scv, allocMemory []uint64, err error)
}

type Yoda struct {
	handle framework.Handle
	gpu    *yodagpu.Handle
	source SnapshotSource
	mode   yodagpu.Mode
	mu     sync.Mutex // one scheduling cycle at a time uses the GPU handle
}

type rowState struct{ row *yodagpu.Row }

func (r *rowState) Clone() framework.StateData { return r }

const rowKey = Name + "/row"

func (y *Yoda) Name() string { return Name }

func NewWithSource(_ runtime.Object, h framework.Handle, src SnapshotSource) (framework.Plugin, error) {
	g, err := yodagpu.New(0)
	if err != nil {
		return nil, err
	}
	return &Yoda{handle: h, gpu: g, source: src, mode: yodagpu.ModeSCV}, nil
}

// Less keeps sort.go:8-10: higher scv/priority first.
func (y *Yoda) Less(a, b *framework.QueuedPodInfo) bool {
	return priority(a.Pod) > priority(b.Pod)
}

// PreFilter refreshes the snapshot if needed and evaluates the whole row on the GPU.
func (y *Yoda) PreFilter(ctx context.Context, state *framework.CycleState, p *v1.Pod) *framework.Status {
	y.mu.Lock()
	defer y.mu.Unlock()
	names, scvs, alloc, err := y.source.Snapshot()
	if err != nil {
		return framework.NewStatus(framework.Error, err.Error())
	}
	if err := y.gpu.UploadNodes(names, scvs, alloc, nil, nil); err != nil {
		return framework.NewStatus(framework.Error, err.Error())
	}
	row, err := y.gpu.ScoreRow(p, y.mode)
	if err != nil {
		return framework.NewStatus(framework.Error, err.Error())
	}
	state.Write(rowKey, &rowState{row})
	return framework.NewStatus(framework.Success, "")
}

func (y *Yoda) PreFilterExtensions() framework.PreFilterExtensions { return nil }

func (y *Yoda) row(state *framework.CycleState) (*yodagpu.Row, error) {
	d, err := state.Read(rowKey)
	if err != nil {
		return nil, err
	}
	return d.(*rowState).row, nil
}

// Filter = PodFitsNumber ∧ PodFitsMemory ∧ PodFitsClock (filter.go:11-58), from the row.
func (y *Yoda) Filter(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	nodeInfo *framework.NodeInfo) *framework.Status {
	row, err := y.row(state)
	if err != nil {
		return framework.NewStatus(framework.Error, err.Error())
	}
	i, ok := y.gpu.NodeIndex(nodeInfo.Node().GetName())
	if !ok || row.Feasible[i/32]>>(uint(i)%32)&1 == 0 {
		return framework.NewStatus(framework.Unschedulable, "node(s) didn't match the scv card requirements")
	}
	return framework.NewStatus(framework.Success, "")
}

func (y *Yoda) PreScore(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	nodes []*v1.Node) *framework.Status {
	return framework.NewStatus(framework.Success, "")
}

// Score returns CalculateBasicScore + Allocate + Actual after Uint64ToInt64 (scheduler.go:154).
func (y *Yoda) Score(ctx context.Context, state *framework.CycleState, p *v1.Pod,
	nodeName string) (int64, *framework.Status) {
	row, err := y.row(state)
	if err != nil {
		return 0, framework.NewStatus(framework.Error, err.Error())
	}
	i, ok := y.gpu.NodeIndex(nodeName)
	if !ok {
		return 0, framework.NewStatus(framework.Error, fmt.Sprintf("node %q not in snapshot", nodeName))
	}
	return row.Score[i], framework.NewStatus(framework.Success, "")
}

func (y *Yoda) ScoreExtensions() framework.ScoreExtensions { return y }

// NormalizeScore: min/max rescale to [0, MaxNodeScore] with the reference's semantics
// (highest starts at 0, lowest at the first score, lowest-- when they are equal).
func (y *Yoda) NormalizeScore(ctx context.Context, state *framework.CycleState, p *v1.Pod,
	scores framework.NodeScoreList) *framework.Status {
	var highest int64
	lowest := scores[0].Score
	for _, s := range scores {
		if s.Score > highest {
			highest = s.Score
		}
		if s.Score < lowest {
			lowest = s.Score
		}
	}
	if highest == lowest {
		lowest--
	}
	for i := range scores {
		scores[i].Score = (scores[i].Score - lowest) * framework.MaxNodeScore / (highest - lowest)
	}
	return framework.NewStatus(framework.Success, "")
}

func (y *Yoda) PreBind(ctx context.Context, state *framework.CycleState, p *v1.Pod,
	nodeName string) *framework.Status {
	if _, err := y.handle.SnapshotSharedLister().NodeInfos().Get(nodeName); err != nil {
		return framework.NewStatus(framework.Error, fmt.Sprintf("prebind get node info error: %+v", nodeName))
	}
	return framework.NewStatus(framework.Success, "")
}

func priority(p *v1.Pod) int {
	if v, ok := p.Labels["scv/priority"]; ok {
		pri, _ := strconvAtoi(v)
		return pri
	}
	return 0
}
