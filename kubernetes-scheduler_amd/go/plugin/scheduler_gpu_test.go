package yoda

// Host-side bookkeeping of the drop-in, no GPU needed:
//
//	go test ./pkg/yoda/ -run Allocated
//
// NOT COMPILED HERE (no Go toolchain in the build image); see INTEGRATION.md.

import (
	"fmt"
	"testing"

	v1 "k8s.io/api/core/v1"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/kubernetes/pkg/scheduler/framework"
)

// fakeLister serves a fixed set of NodeInfos as the scheduler's snapshot.
type fakeLister struct{ infos map[string]*framework.NodeInfo }

func (f fakeLister) NodeInfos() framework.NodeInfoLister { return f }
func (f fakeLister) List() ([]*framework.NodeInfo, error) {
	out := make([]*framework.NodeInfo, 0, len(f.infos))
	for _, ni := range f.infos {
		out = append(out, ni)
	}
	return out, nil
}
func (f fakeLister) HavePodsWithAffinityList() ([]*framework.NodeInfo, error) { return nil, nil }
func (f fakeLister) HavePodsWithRequiredAntiAffinityList() ([]*framework.NodeInfo, error) {
	return nil, nil
}
func (f fakeLister) Get(name string) (*framework.NodeInfo, error) {
	if ni, ok := f.infos[name]; ok {
		return ni, nil
	}
	return nil, fmt.Errorf("node %q not found", name)
}

// fakeHandle: only SnapshotSharedLister is called by allocated (the embedded nil Handle
// panics on anything else).
type fakeHandle struct {
	framework.Handle
	l fakeLister
}

func (h fakeHandle) SnapshotSharedLister() framework.SharedLister { return h.l }

func memPod(name, mem string) *v1.Pod {
	return &v1.Pod{ObjectMeta: metav1.ObjectMeta{Name: name, Labels: map[string]string{"scv/memory": mem}}}
}

func nodeInfo(name string, pods ...*v1.Pod) *framework.NodeInfo {
	ni := framework.NewNodeInfo(pods...)
	ni.SetNode(&v1.Node{ObjectMeta: metav1.ObjectMeta{Name: name}})
	return ni
}

// allocated sums the scv/memory labels per node (algorithm.go:299-303), reuses the sums of
// nodes whose NodeInfo generation did not move, and re-walks a node once a pod is added.
func TestAllocatedFollowsGenerations(t *testing.T) {
	a := nodeInfo("a", memPod("p1", "100"), memPod("p2", "23"))
	b := nodeInfo("b")
	l := fakeLister{infos: map[string]*framework.NodeInfo{"a": a, "b": b}}
	y := &Yoda{handle: fakeHandle{l: l}}
	names := []string{"a", "b", "gone"}
	alloc, gens := y.allocated(names, nil, nil)
	if alloc[0] != 123 || alloc[1] != 0 || alloc[2] != 0 || gens[2] != -1 {
		t.Fatalf("first pass: alloc %v gens %v", alloc, gens)
	}
	// an unchanged generation keeps the previous sum (a stale value proves no re-walk)
	stale := []uint64{7, 0, 0}
	again, _ := y.allocated(names, stale, gens)
	if again[0] != 7 {
		t.Fatalf("unchanged generation re-walked node a: %v", again)
	}
	// the scheduler assumes a pod on b: its generation moves, its sum is recomputed
	b.AddPod(memPod("p3", "40"))
	after, gens2 := y.allocated(names, again, gens)
	if after[1] != 40 || gens2[1] == gens[1] || after[0] != 7 {
		t.Fatalf("after AddPod: alloc %v gens %v -> %v", after, gens, gens2)
	}
}

// Mode B's node set (snapshotNodes): every node of the scheduler's snapshot, in name order,
// NodeInfos without a Node skipped -- the nodes the reference's pass-through Filter hands to
// PreScore (scheduler.go:96-99,122), uploaded with the advisor's metrics each cycle.
func TestModeBSnapshotNodes(t *testing.T) {
	orphan := framework.NewNodeInfo() // no Node set (a NodeInfo the cache holds pods for)
	l := fakeLister{infos: map[string]*framework.NodeInfo{
		"n2": nodeInfo("n2"), "n10": nodeInfo("n10"), "n1": nodeInfo("n1"), "x": orphan,
	}}
	y := &Yoda{handle: fakeHandle{l: l}}
	names, err := y.snapshotNodes()
	if err != nil {
		t.Fatal(err)
	}
	want := []string{"n1", "n10", "n2"}
	if fmt.Sprint(names) != fmt.Sprint(want) {
		t.Fatalf("snapshotNodes = %v, want %v", names, want)
	}
}

// Less keeps sort.go:8-18: higher scv/priority first; a missing or non-numeric label is 0
// (Atoi error -> 0), a negative one stays negative.
func TestLessFollowsScvPriority(t *testing.T) {
	pod := func(p string) *framework.QueuedPodInfo {
		labels := map[string]string{}
		if p != "" {
			labels["scv/priority"] = p
		}
		return &framework.QueuedPodInfo{PodInfo: framework.NewPodInfo(
			&v1.Pod{ObjectMeta: metav1.ObjectMeta{Name: "p" + p, Labels: labels}})}
	}
	y := &Yoda{}
	cases := []struct {
		a, b string
		less bool
	}{{"5", "3", true}, {"3", "5", false}, {"1", "", true}, {"", "x", false}, {"-1", "", false},
		{"", "-1", true}, {"7", "7", false}}
	for _, c := range cases {
		if got := y.Less(pod(c.a), pod(c.b)); got != c.less {
			t.Errorf("Less(%q, %q) = %v, want %v", c.a, c.b, got, c.less)
		}
	}
}
