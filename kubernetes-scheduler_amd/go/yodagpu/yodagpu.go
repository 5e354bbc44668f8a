// Package yodagpu binds libyoda (include/yoda.h) through cgo for the Yoda kube-scheduler
// plugin (github.com/Mr-LvGJ/Yoda-Scheduler/pkg/yoda).  It is the Go half of the drop-in
// boundary documented in INTEGRATION.md.
//
// NOT COMPILED IN THIS REPOSITORY'S CI: the build image has no Go toolchain.  The C-ABI it
// calls is exercised from C (tools/capi_example.c) and Python ctypes (yoda_amd/capi.py).
package yodagpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../yoda_amd -lyoda -Wl,-rpath,${SRCDIR}/../../yoda_amd
#include <stdlib.h>
#include "yoda.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"unsafe"

	scv "github.com/NJUPT-ISL/SCV/api/v1"
	v1 "k8s.io/api/core/v1"

	"github.com/Mr-LvGJ/Yoda-Scheduler/pkg/yoda/filter"
	"github.com/Mr-LvGJ/Yoda-Scheduler/pkg/yoda/score"
)

// Mode selects the score: the SCV GPU path (Mode A) or the shipped diskIO balance (Mode B).
type Mode int

const (
	ModeSCV    Mode = C.YODA_MODE_SCV
	ModeDiskIO Mode = C.YODA_MODE_DISKIO
)

// Handle owns one libyoda handle (one GPU, one node snapshot).  Not safe for concurrent
// use: the framework calls PreFilter once per pod cycle, cycles are serial.
type Handle struct {
	h     *C.yoda_t
	nodes []string
	index map[string]int
}

func check(h *C.yoda_t, rc C.int, what string) error {
	if rc == C.YODA_OK {
		return nil
	}
	msg := ""
	if h != nil {
		msg = C.GoString(C.yoda_last_error(h))
	}
	return fmt.Errorf("%s: libyoda error %d: %s", what, int(rc), msg)
}

// New opens a handle on GPU `device`.
func New(device int) (*Handle, error) {
	var h *C.yoda_t
	if err := check(nil, C.yoda_create(C.int(device), &h), "yoda_create"); err != nil {
		return nil, err
	}
	g := &Handle{h: h}
	runtime.SetFinalizer(g, (*Handle).Close)
	return g, nil
}

// Close releases the device memory.
func (g *Handle) Close() {
	if g.h != nil {
		C.yoda_destroy(g.h)
		g.h = nil
	}
}

// cArray pins a Go slice for the duration of a call (cgo pointer rules: the C side keeps
// no reference after returning).
func u64p(s []uint64) *C.uint64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint64_t)(unsafe.Pointer(&s[0]))
}
func u32p(s []uint32) *C.uint32_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint32_t)(unsafe.Pointer(&s[0]))
}
func u8p(s []uint8) *C.uint8_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&s[0]))
}
func f64p(s []float64) *C.double {
	if len(s) == 0 {
		return nil
	}
	return (*C.double)(unsafe.Pointer(&s[0]))
}
func i64p(s []int64) *C.int64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.int64_t)(unsafe.Pointer(&s[0]))
}

// UploadNodes packs the SCV records (one per node, in the order of `names`) into the
// struct-of-arrays of yoda_node_soa and uploads them.  allocMemory[i] is the sum of the
// scv/memory labels of pods already on node i (score.CalculateAllocateScore's loop,
// algorithm.go:299-303); cpu/diskIO are advisor.NodeInfo values (Mode B, may be nil).
func (g *Handle) UploadNodes(names []string, scvs []*scv.Scv, allocMemory []uint64,
	cpu, diskIO []float64) error {
	n := len(scvs)
	k := 1
	for _, s := range scvs {
		if len(s.Status.CardList) > k {
			k = len(s.Status.CardList)
		}
	}
	if k > C.YODA_MAX_CARDS {
		return errors.New("more than YODA_MAX_CARDS cards on a node")
	}
	cardNumber := make([]uint64, n)
	cardCount := make([]uint32, n)
	freeSum := make([]uint64, n)
	totalSum := make([]uint64, n)
	free := make([]uint64, n*k)
	total := make([]uint64, n*k)
	clock := make([]uint64, n*k)
	bw := make([]uint64, n*k)
	core := make([]uint64, n*k)
	power := make([]uint64, n*k)
	healthy := make([]uint8, n*k)
	for i, s := range scvs {
		cardNumber[i] = uint64(s.Status.CardNumber)
		cardCount[i] = uint32(len(s.Status.CardList))
		freeSum[i] = s.Status.FreeMemorySum
		totalSum[i] = s.Status.TotalMemorySum
		for j, c := range s.Status.CardList {
			o := i*k + j
			free[o], total[o] = c.FreeMemory, c.TotalMemory
			clock[o], bw[o] = uint64(c.Clock), uint64(c.Bandwidth)
			core[o], power[o] = uint64(c.Core), uint64(c.Power)
			if c.Health == "Healthy" { // filter.go:53,57
				healthy[o] = 1
			}
		}
	}
	soa := C.yoda_node_soa{
		n_nodes: C.uint32_t(n), max_cards: C.uint32_t(k),
		card_number: u64p(cardNumber), card_count: u32p(cardCount),
		free_memory_sum: u64p(freeSum), total_memory_sum: u64p(totalSum),
		alloc_memory:     u64p(allocMemory),
		card_free_memory: u64p(free), card_total_memory: u64p(total),
		card_clock: u64p(clock), card_bandwidth: u64p(bw), card_core: u64p(core),
		card_power: u64p(power), card_healthy: u8p(healthy),
		cpu: f64p(cpu), disk_io: f64p(diskIO),
	}
	if err := check(g.h, C.yoda_upload_nodes(g.h, &soa, 0, 0), "yoda_upload_nodes"); err != nil {
		return err
	}
	g.nodes = names
	g.index = make(map[string]int, len(names))
	for i, name := range names {
		g.index[name] = i
	}
	return nil
}

// PackPods parses the scv/* labels and the diskIO annotation with the reference's own
// helpers (filter.go:60-74, sort.go:12-18, algorithm.go:103-104) into yoda_pod_soa arrays.
type PodBatch struct {
	hasNumber, hasMemory, hasClock []uint8
	number, memory, clock          []uint64
	priority, rcpu                 []int64
	rio                            []float64
}

func PackPods(pods []*v1.Pod) *PodBatch {
	b := &PodBatch{}
	for _, p := range pods {
		l := p.GetLabels()
		has := func(key string) (uint8, uint64) {
			if v, ok := l[key]; ok {
				return 1, filter.StrToUint64(v)
			}
			return 0, 0
		}
		hn, n := has("scv/number")
		hm, m := has("scv/memory")
		hc, c := has("scv/clock")
		b.hasNumber, b.number = append(b.hasNumber, hn), append(b.number, n)
		b.hasMemory, b.memory = append(b.hasMemory, hm), append(b.memory, m)
		b.hasClock, b.clock = append(b.hasClock, hc), append(b.clock, c)
		prio := int64(0)
		if v, ok := l["scv/priority"]; ok {
			pr, _ := strconvAtoi(v)
			prio = int64(pr)
		}
		b.priority = append(b.priority, prio)
		rio, _ := strconvParseFloat32(p.Annotations["diskIO"])
		b.rio = append(b.rio, rio)
		b.rcpu = append(b.rcpu, score.CalculatePodResourceRequest(p, v1.ResourceCPU, true))
	}
	return b
}

func (b *PodBatch) soa() C.yoda_pod_soa {
	return C.yoda_pod_soa{
		n_pods:     C.uint32_t(len(b.number)),
		has_number: u8p(b.hasNumber), number: u64p(b.number),
		has_memory: u8p(b.hasMemory), memory: u64p(b.memory),
		has_clock: u8p(b.hasClock), clock: u64p(b.clock),
		priority: i64p(b.priority), rio: f64p(b.rio), rcpu: i64p(b.rcpu),
	}
}

// Row is one pod's Filter result and raw Score for every node of the snapshot.
type Row struct {
	Feasible []uint32 // bitmask, bit (n & 31) of word n/32
	Score    []int64  // Yoda.Score's value (after Uint64ToInt64); -1 where Filter fails
}

// ScoreRow evaluates ONE pod against every node: the plugin's PreFilter calls it once per
// scheduling cycle, so Filter and Score become lookups.
func (g *Handle) ScoreRow(pod *v1.Pod, mode Mode) (*Row, error) {
	b := PackPods([]*v1.Pod{pod})
	s := b.soa()
	if err := check(g.h, C.yoda_upload_pods(g.h, &s), "yoda_upload_pods"); err != nil {
		return nil, err
	}
	n := len(g.nodes)
	row := &Row{Feasible: make([]uint32, (n+31)/32), Score: make([]int64, n)}
	rc := C.yoda_score_rows(g.h, C.int(mode), u32p(row.Feasible), C.uint64_t(len(row.Feasible)),
		i64p(row.Score), C.uint64_t(n))
	if err := check(g.h, rc, "yoda_score_rows"); err != nil {
		return nil, err
	}
	return row, nil
}

// Batch schedules many pods independently against the snapshot (configs 2-4).  Picks are
// node indices, -1 unschedulable, -2 error (see statuses).
func (g *Handle) Batch(pods []*v1.Pod, mode Mode) (picks []int32, statuses []int32, err error) {
	b := PackPods(pods)
	s := b.soa()
	picks = make([]int32, len(pods))
	statuses = make([]int32, len(pods))
	out := C.yoda_eval_out{
		pick:   (*C.int32_t)(unsafe.Pointer(&picks[0])),
		status: (*C.int32_t)(unsafe.Pointer(&statuses[0])),
	}
	err = check(g.h, C.yoda_eval(g.h, &s, C.int(mode), &out), "yoda_eval")
	return
}

// Greedy schedules the pods one after another in sort.Less order, each pick updating the
// node's Allocate score (config 5).
func (g *Handle) Greedy(pods []*v1.Pod, mode Mode, cardCapacity bool) ([]int32, error) {
	b := PackPods(pods)
	s := b.soa()
	picks := make([]int32, len(pods))
	flags := C.uint32_t(0)
	if cardCapacity {
		flags = C.YODA_GREEDY_CARD_CAPACITY
	}
	rc := C.yoda_greedy(g.h, &s, C.int(mode), flags, (*C.int32_t)(unsafe.Pointer(&picks[0])))
	return picks, check(g.h, rc, "yoda_greedy")
}

// NodeIndex maps a node name to its row position.
func (g *Handle) NodeIndex(name string) (int, bool) {
	i, ok := g.index[name]
	return i, ok
}
