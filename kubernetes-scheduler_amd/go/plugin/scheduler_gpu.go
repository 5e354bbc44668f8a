// Package yoda — the GPU-backed Yoda plugin: a drop-in for pkg/yoda/scheduler.go of
// Mr-LvGJ/kubernetes-scheduler, served by libyoda through yodagpu.  Placed in pkg/yoda in
// place of scheduler.go, it keeps the package name, Name and the factory signature, so the
// registration compiles unchanged (pkg/register/register.go:8-12):
//
//	app.NewSchedulerCommand(app.WithPlugin(yoda.Name, yoda.New))
//
// Per scheduling cycle PreFilter brings the device snapshot up to date and evaluates the
// pod against EVERY node in one libyoda call (Filter, PreScore maxima, Score); Filter and
// Score are then lookups, NormalizeScore is the reference's code (scheduler.go:158-183).
//
// NOT COMPILED HERE (no Go toolchain in the build image); see INTEGRATION.md.
package yoda

import (
	"context"
	"fmt"
	"sort"
	"strconv"
	"sync"
	"sync/atomic"

	scv "github.com/NJUPT-ISL/SCV/api/v1"
	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/apis/meta/v1/unstructured"
	"k8s.io/apimachinery/pkg/labels"
	"k8s.io/apimachinery/pkg/runtime"
	"k8s.io/apimachinery/pkg/runtime/schema"
	"k8s.io/client-go/dynamic"
	"k8s.io/client-go/dynamic/dynamicinformer"
	toolscache "k8s.io/client-go/tools/cache"
	"k8s.io/klog/v2"
	"k8s.io/kubernetes/pkg/scheduler/framework"
	frameworkruntime "k8s.io/kubernetes/pkg/scheduler/framework/runtime"

	"github.com/Mr-LvGJ/Yoda-Scheduler/pkg/yoda/advisor"
	"github.com/Mr-LvGJ/Yoda-Scheduler/pkg/yoda/filter"
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

// Args keeps the reference's (cosmetic) fields, so existing KubeSchedulerConfiguration
// pluginConfig entries still decode (scheduler.go:36-40, deploy/yoda-scheduler.yaml:42-47),
// and adds the GPU plugin's own:
//
//	mode    "scv" (default): the SCV GPU score (filter.go + collection.go + algorithm.go:
//	        264-310, the north-star path); "diskio": BalancedCpuDiskIOPriority
//	        (algorithm.go:99-119), what the reference binary scores, with Filter a
//	        pass-through and the node metrics from the reference's own advisor (Prometheus).
//	device  the GPU ordinal.
type Args struct {
	FavoriteColor  string `json:"favorite_color,omitempty"`
	FavoriteNumber int    `json:"favorite_number,omitempty"`
	ThanksTo       string `json:"thanks_to,omitempty"`
	Mode           string `json:"mode,omitempty"`
	Device         int    `json:"device,omitempty"`
}

// SnapshotSource gives the SCV records (core.run-linux.com/v1 scvs, deploy/yoda-scheduler.yaml:
// 225-236) in node order and a generation that changes whenever any record does.
type SnapshotSource interface {
	SCVs() (names []string, scvs []*scv.Scv, gen uint64, err error)
}

type Yoda struct {
	handle framework.Handle
	gpu    *yodagpu.Handle
	source SnapshotSource
	mode   yodagpu.Mode
	mu     sync.Mutex // one scheduling cycle at a time uses the GPU handle

	loaded     bool
	gen        uint64   // generation of the uploaded SCV records
	alloc      []uint64 // allocated scv/memory per node as on the device
	cardNumber []uint64
}

type rowState struct{ row *yodagpu.Row }

func (r *rowState) Clone() framework.StateData { return r }

const rowKey = Name + "/row"

func (y *Yoda) Name() string { return Name }

// New is the plugin factory registered by pkg/register (scheduler.go:57's signature).
func New(obj runtime.Object, h framework.Handle) (framework.Plugin, error) {
	args := &Args{}
	if obj != nil {
		if err := frameworkruntime.DecodeInto(obj, args); err != nil {
			return nil, err
		}
	}
	klog.V(3).Infof("yoda (GPU) plugin args: %+v", args)
	src, err := NewInformerSource(h)
	if err != nil {
		return nil, err
	}
	return NewWithSource(args, h, src)
}

// NewWithSource builds the plugin over any SnapshotSource (tests, file-backed snapshots).
func NewWithSource(args *Args, h framework.Handle, src SnapshotSource) (*Yoda, error) {
	mode := yodagpu.ModeSCV
	switch args.Mode {
	case "", "scv":
	case "diskio":
		mode = yodagpu.ModeDiskIO
	default:
		return nil, fmt.Errorf("yoda: unknown mode %q (want scv or diskio)", args.Mode)
	}
	g, err := yodagpu.New(args.Device)
	if err != nil {
		return nil, err
	}
	return &Yoda{handle: h, gpu: g, source: src, mode: mode}, nil
}

// ---- SCV records from an informer ---------------------------------------------------------

var scvGVR = schema.GroupVersionResource{Group: "core.run-linux.com", Version: "v1",
	Resource: "scvs"}

type informerSource struct {
	lister toolscache.GenericLister
	gen    uint64 // bumped by every add / update / delete (atomic)
}

// NewInformerSource watches the SCV custom resources through a dynamic shared informer
// (the RBAC of deploy/yoda-scheduler.yaml:225-236 already grants get/list/watch on them).
func NewInformerSource(h framework.Handle) (SnapshotSource, error) {
	dc, err := dynamic.NewForConfig(h.KubeConfig())
	if err != nil {
		return nil, err
	}
	f := dynamicinformer.NewDynamicSharedInformerFactory(dc, 0)
	inf := f.ForResource(scvGVR)
	s := &informerSource{lister: inf.Lister()}
	bump := func(interface{}) { atomic.AddUint64(&s.gen, 1) }
	inf.Informer().AddEventHandler(toolscache.ResourceEventHandlerFuncs{
		AddFunc:    bump,
		UpdateFunc: func(_, o interface{}) { bump(o) },
		DeleteFunc: bump,
	})
	stop := make(chan struct{}) // lives as long as the scheduler process
	f.Start(stop)
	f.WaitForCacheSync(stop)
	return s, nil
}

func (s *informerSource) SCVs() ([]string, []*scv.Scv, uint64, error) {
	gen := atomic.LoadUint64(&s.gen) // read first: a later change shows up next cycle
	objs, err := s.lister.List(labels.Everything())
	if err != nil {
		return nil, nil, 0, err
	}
	out := make([]*scv.Scv, 0, len(objs))
	for _, o := range objs {
		u, ok := o.(*unstructured.Unstructured)
		if !ok {
			continue
		}
		x := &scv.Scv{}
		if err := runtime.DefaultUnstructuredConverter.FromUnstructured(u.Object, x); err != nil {
			return nil, nil, 0, err
		}
		out = append(out, x)
	}
	sort.Slice(out, func(i, j int) bool { return out[i].Name < out[j].Name })
	names := make([]string, len(out))
	for i, x := range out {
		names[i] = x.Name
	}
	return names, out, gen, nil
}

// ---- the device snapshot --------------------------------------------------------------------

// allocated returns, per snapshot node, the sum of the scv/memory labels of the pods the
// scheduler's snapshot has on it -- assumed pods included, as in CalculateAllocateScore's
// loop over nodeInfo.Pods (algorithm.go:299-303).
func (y *Yoda) allocated(names []string) []uint64 {
	alloc := make([]uint64, len(names))
	infos := y.handle.SnapshotSharedLister().NodeInfos()
	for i, n := range names {
		ni, err := infos.Get(n)
		if err != nil {
			continue // an SCV record without a schedulable node: nothing allocated on it
		}
		for _, pi := range ni.Pods {
			if mem, ok := pi.Pod.GetLabels()["scv/memory"]; ok {
				alloc[i] += filter.StrToUint64(mem)
			}
		}
	}
	return alloc
}

// refresh brings the device snapshot up to date: a full upload when the SCV records
// changed (or every cycle in Mode B, whose node metrics come from Prometheus each cycle as in
// the reference's PreScore, scheduler.go:101-114); otherwise only the nodes whose allocated
// memory moved since the last cycle (the scheduler's assumes and binds) are pushed.
func (y *Yoda) refresh() error {
	names, scvs, gen, err := y.source.SCVs()
	if err != nil {
		return err
	}
	alloc := y.allocated(names)
	if y.mode == yodagpu.ModeDiskIO || !y.loaded || gen != y.gen {
		var cpu, disk []float64
		if y.mode == yodagpu.ModeDiskIO {
			info, err := advisor.Result{}.Init() // advisor.go:149-265
			if err != nil {
				return err
			}
			cpu, disk = make([]float64, len(names)), make([]float64, len(names))
			for i, n := range names {
				ni, ok := info.Info[n]
				if !ok {
					// the reference dereferences a nil NodeInfo here (algorithm.go:70,73)
					return fmt.Errorf("node %q missing from the advisor's metrics", n)
				}
				cpu[i], disk[i] = ni.Cpu, ni.DiskIO
			}
		}
		if err := y.gpu.UploadNodes(names, scvs, alloc, cpu, disk); err != nil {
			return err
		}
		y.loaded, y.gen, y.alloc = true, gen, alloc
		y.cardNumber = make([]uint64, len(scvs))
		for i, s := range scvs {
			y.cardNumber[i] = uint64(s.Status.CardNumber)
		}
		return nil
	}
	var idx []uint32
	var al, cn []uint64
	for i := range alloc {
		if alloc[i] != y.alloc[i] {
			idx = append(idx, uint32(i))
			al = append(al, alloc[i])
			cn = append(cn, y.cardNumber[i])
		}
	}
	if err := y.gpu.SetNodeState(idx, al, cn); err != nil {
		return err
	}
	y.alloc = alloc
	return nil
}

// ---- extension points -----------------------------------------------------------------------

// Less keeps sort.go:8-10: higher scv/priority first.
func (y *Yoda) Less(a, b *framework.QueuedPodInfo) bool {
	return priority(a.Pod) > priority(b.Pod)
}

// PreFilter refreshes the snapshot if needed and evaluates the whole row on the GPU.
func (y *Yoda) PreFilter(ctx context.Context, state *framework.CycleState, p *v1.Pod) *framework.Status {
	y.mu.Lock()
	defer y.mu.Unlock()
	if err := y.refresh(); err != nil {
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

// Filter = PodFitsNumber ∧ PodFitsMemory ∧ PodFitsClock (filter.go:11-58), from the row
// (Mode B: every node, as the reference's pass-through Filter, scheduler.go:96-99).
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
// A node with TotalMemorySum == 0 is a framework Error: the reference divides by it
// (algorithm.go:294,309) and panics.  k8s does not call Score when only one node passed
// Filter, so that case never reaches here.
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
	if y.mode == yodagpu.ModeSCV && y.gpu.ZeroTotal(i) {
		return 0, framework.NewStatus(framework.Error,
			fmt.Sprintf("node %q: TotalMemorySum is 0 (integer divide by zero in the reference score)", nodeName))
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
		pri, _ := strconv.Atoi(v) // sort.GetPodPriority (sort.go:12-18)
		return pri
	}
	return 0
}
