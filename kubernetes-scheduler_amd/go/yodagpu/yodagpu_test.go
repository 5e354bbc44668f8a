package yodagpu

// Run on a machine with Go, libyoda.so built and an MI355X:
//
//	GODEBUG=cgocheck=1 go test ./pkg/yoda/yodagpu/
//
// cgocheck=1 (the default) panics on the first cgo call that passes a Go pointer to Go
// memory holding Go pointers; every call below goes through the structs of yoda.h.

import (
	"testing"

	scv "github.com/NJUPT-ISL/SCV/api/v1"
	v1 "k8s.io/api/core/v1"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
)

// KAT 1 of SURVEY.md §8c: pick = node1, raw scores 1718 / 4061, node2 infeasible.
func kat1() ([]string, []*scv.Scv, []uint64, *v1.Pod) {
	card := func(h string, free, total uint64, clock, bw, core, power uint) scv.Card {
		return scv.Card{Health: h, FreeMemory: free, TotalMemory: total, Clock: clock,
			Bandwidth: bw, Core: core, Power: power}
	}
	n0 := &scv.Scv{}
	n0.Status.CardNumber = 2
	n0.Status.CardList = []scv.Card{card("Healthy", 10000, 16000, 1500, 900, 80, 300),
		card("Healthy", 9000, 16000, 1500, 900, 80, 300)}
	n0.Status.FreeMemorySum, n0.Status.TotalMemorySum = 19000, 32000
	n1 := &scv.Scv{}
	n1.Status.CardNumber = 4
	c1 := card("Healthy", 16000, 32000, 1500, 1200, 108, 400)
	n1.Status.CardList = []scv.Card{c1, c1, c1, card("Unhealthy", 16000, 32000, 1500, 1200, 108, 400)}
	n1.Status.FreeMemorySum, n1.Status.TotalMemorySum = 64000, 128000
	n2 := &scv.Scv{}
	n2.Status.CardNumber = 1
	n2.Status.CardList = []scv.Card{card("Healthy", 16000, 32000, 1500, 1200, 108, 400)}
	n2.Status.FreeMemorySum, n2.Status.TotalMemorySum = 16000, 32000
	pod := &v1.Pod{ObjectMeta: metav1.ObjectMeta{Name: "p", Labels: map[string]string{
		"scv/number": "2", "scv/memory": "8000", "scv/clock": "1500"}}}
	return []string{"node0", "node1", "node2"}, []*scv.Scv{n0, n1, n2}, []uint64{0, 16000, 0}, pod
}

func TestScoreRowKAT1(t *testing.T) {
	g, err := New(0)
	if err != nil {
		t.Skipf("no GPU / libyoda: %v", err)
	}
	defer g.Close()
	names, scvs, alloc, pod := kat1()
	if err := g.UploadNodes(names, scvs, alloc, nil, nil); err != nil {
		t.Fatal(err)
	}
	row, err := g.ScoreRow(pod, ModeSCV)
	if err != nil {
		t.Fatal(err)
	}
	if row.Feasible[0] != 0b011 || row.Score[0] != 1718 || row.Score[1] != 4061 || row.Score[2] != -1 {
		t.Fatalf("row = %b %v", row.Feasible[0], row.Score)
	}
	picks, st, err := g.Batch([]*v1.Pod{pod, pod}, ModeSCV)
	if err != nil || picks[0] != 1 || picks[1] != 1 || st[0] != StatusOK {
		t.Fatalf("batch = %v %v %v", picks, st, err)
	}
	// the assume of a pod on node1 through the sparse node-state push
	if err := g.SetNodeState([]uint32{1}, []uint64{16000 + 8000}, []uint64{4}); err != nil {
		t.Fatal(err)
	}
	if row, err = g.ScoreRow(pod, ModeSCV); err != nil || row.Score[1] >= 4061 {
		t.Fatalf("after assume: %v %v", row.Score, err)
	}
	// empty batches are no-ops, not index panics
	if p, s, err := g.Batch(nil, ModeSCV); p != nil || s != nil || err != nil {
		t.Fatal("empty Batch")
	}
	if p, err := g.Greedy(nil, ModeSCV, true); p != nil || err != nil {
		t.Fatal("empty Greedy")
	}
}
