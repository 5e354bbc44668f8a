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
	"time"

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
	source SnapshotSource // SCV records (Mode A); nil in Mode B
	mode   yodagpu.Mode
	mu     sync.Mutex // one scheduling cycle at a time uses the GPU handle

	loaded     bool
	gen        uint64   // generation of the uploaded SCV records
	names      []string // the uploaded node order
	alloc      []uint64 // allocated scv/memory per node as on the device
	nodeGen    []int64  // framework.NodeInfo.Generation each alloc[i] was summed at (-1: none)
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
	if args.Mode == "diskio" { // Mode B scores the snapshot's nodes: no SCV records needed
		return NewWithSource(args, h, nil)
	}
	src, err := NewInformerSource(h, cacheSyncTimeout)
	if err != nil {
		return nil, err
	}
	return NewWithSource(args, h, src)
}

// cacheSyncTimeout bounds the wait for the SCV informer's first list: a missing CRD or RBAC
// that denies list/watch then fails the plugin factory instead of hanging the scheduler.
const cacheSyncTimeout = 60 * time.Second

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
// (the RBAC of deploy/yoda-scheduler.yaml:225-236 already grants get/list/watch on them).  It
// returns an error when the informer has not synced within `timeout`.
func NewInformerSource(h framework.Handle, timeout time.Duration) (SnapshotSource, error) {
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
	wait := make(chan struct{}) // closes at the deadline: WaitForCacheSync gives up then
	timer := time.AfterFunc(timeout, func() { close(wait) })
	defer timer.Stop()
	for gvr, ok := range f.WaitForCacheSync(wait) {
		if !ok {
			close(stop)
			return nil, fmt.Errorf("yoda: the %s informer did not sync within %v (is the SCV CRD "+
				"installed, and may the scheduler list/watch it?)", gvr.Resource, timeout)
		}
	}
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

// podMemory is CalculateAllocateScore's sum for one node: the scv/memory labels of the pods
// the scheduler's snapshot has on it, assumed pods included (algorithm.go:299-303).
func podMemory(ni *framework.NodeInfo) uint64 {
	var sum uint64
	for _, pi := range ni.Pods {
		if mem, ok := pi.Pod.GetLabels()["scv/memory"]; ok {
			sum += filter.StrToUint64(mem) // uint64 wrap, as the reference
		}
	}
	return sum
}

// allocated returns, per node of `names`, podMemory of its snapshot NodeInfo, and the
// NodeInfo generations it was summed at.  prev/prevGen (same node order, may be nil): a node
// whose generation did not move keeps its previous sum -- the framework bumps
// NodeInfo.Generation on every pod added to or removed from the node, so a cycle walks the
// pods of the changed nodes only, not every pod of the cluster.
func (y *Yoda) allocated(names []string, prev []uint64, prevGen []int64) ([]uint64, []int64) {
	alloc := make([]uint64, len(names))
	gens := make([]int64, len(names))
	infos := y.handle.SnapshotSharedLister().NodeInfos()
	for i, n := range names {
		gens[i] = -1
		ni, err := infos.Get(n)
		if err != nil {
			continue // an SCV record without a schedulable node: nothing allocated on it
		}
		gens[i] = ni.Generation
		if prev != nil && prevGen[i] == ni.Generation {
			alloc[i] = prev[i]
			continue
		}
		alloc[i] = podMemory(ni)
	}
	return alloc, gens
}

// snapshotNodes is Mode B's node set: every node of the scheduler's snapshot (the reference's
// Filter passes them all and PreScore scores NodeInfos().List(), scheduler.go:96-99,122).
func (y *Yoda) snapshotNodes() ([]string, error) {
	infos, err := y.handle.SnapshotSharedLister().NodeInfos().List()
	if err != nil {
		return nil, err
	}
	names := make([]string, 0, len(infos))
	for _, ni := range infos {
		if ni.Node() != nil {
			names = append(names, ni.Node().GetName())
		}
	}
	sort.Strings(names)
	return names, nil
}

// refresh brings the device snapshot up to date: a full upload when the SCV records
// changed (or every cycle in Mode B, whose node metrics come from Prometheus each cycle as in
// the reference's PreScore, scheduler.go:101-114); otherwise only the nodes whose allocated
// memory moved since the last cycle (the scheduler's assumes and binds) are pushed.
func (y *Yoda) refresh() error {
	if y.mode == yodagpu.ModeDiskIO {
		// Mode B: the snapshot's nodes, each with the advisor's metrics; a snapshot node the
		// advisor does not report is the reference's nil dereference (algorithm.go:70,73)
		names, err := y.snapshotNodes()
		if err != nil {
			return err
		}
		info, err := advisor.Result{}.Init() // advisor.go:149-265
		if err != nil {
			return err
		}
		cpu, disk := make([]float64, len(names)), make([]float64, len(names))
		for i, n := range names {
			ni, ok := info.Info[n]
			if !ok {
				return fmt.Errorf("node %q missing from the advisor's metrics", n)
			}
			cpu[i], disk[i] = ni.Cpu, ni.DiskIO
		}
		y.names = names
		return y.gpu.UploadNodes(names, nil, nil, cpu, disk)
	}
	names, scvs, gen, err := y.source.SCVs()
	if err != nil {
		return err
	}
	if !y.loaded || gen != y.gen {
		alloc, gens := y.allocated(names, nil, nil)
		if err := y.gpu.UploadNodes(names, scvs, alloc, nil, nil); err != nil {
			return err
		}
		y.loaded, y.gen, y.names, y.alloc, y.nodeGen = true, gen, names, alloc, gens
		y.cardNumber = make([]uint64, len(scvs))
		for i, s := range scvs {
			y.cardNumber[i] = uint64(s.Status.CardNumber)
		}
		return nil
	}
	alloc, gens := y.allocated(y.names, y.alloc, y.nodeGen)
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
	y.alloc, y.nodeGen = alloc, gens
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
