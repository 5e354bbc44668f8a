// Package yodagpu binds libyoda (include/yoda.h) through cgo for the Yoda kube-scheduler
// plugin (github.com/Mr-LvGJ/Yoda-Scheduler/pkg/yoda).  It is the Go half of the drop-in
// boundary documented in INTEGRATION.md.
//
// cgo pointer rules: libyoda's SoA structs (yoda_node_soa, yoda_pod_soa, yoda_eval_out) hold
// pointers, so every array they point at lives in C memory (cArrays below), never in the Go
// heap; a Go pointer is passed to C only directly as an argument, to memory that holds no
// pointers (output slices of plain numbers).  Runs clean under GODEBUG=cgocheck=1
// (yodagpu_test.go).
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
	"strconv"
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

// Status codes of a pod's outcome (include/yoda.h YODA_STATUS_*).
const (
	StatusOK            = C.YODA_STATUS_OK
	StatusUnschedulable = C.YODA_STATUS_UNSCHEDULABLE
	StatusDivZero       = C.YODA_STATUS_DIV_ZERO
	StatusScoreRange    = C.YODA_STATUS_SCORE_RANGE
)

// cArray is a grow-only block of C memory.
type cArray struct {
	p unsafe.Pointer
	n uintptr
}

func (a *cArray) ensure(bytes uintptr) unsafe.Pointer {
	if bytes == 0 {
		bytes = 8
	}
	if bytes > a.n {
		C.free(a.p)
		a.p = C.calloc(1, C.size_t(bytes))
		if a.p == nil {
			panic("yodagpu: out of C memory")
		}
		a.n = bytes
	}
	return a.p
}

func (a *cArray) free() {
	C.free(a.p)
	a.p, a.n = nil, 0
}

// Go views of C memory (Go 1.15-compatible: no unsafe.Slice).
func u64s(a *cArray, n int) []uint64 {
	return (*[1 << 30]uint64)(a.ensure(uintptr(n) * 8))[:n:n]
}
func u32s(a *cArray, n int) []uint32 {
	return (*[1 << 30]uint32)(a.ensure(uintptr(n) * 4))[:n:n]
}
func i64s(a *cArray, n int) []int64 {
	return (*[1 << 30]int64)(a.ensure(uintptr(n) * 8))[:n:n]
}
func i32s(a *cArray, n int) []int32 {
	return (*[1 << 30]int32)(a.ensure(uintptr(n) * 4))[:n:n]
}
func u8s(a *cArray, n int) []uint8 {
	return (*[1 << 31]uint8)(a.ensure(uintptr(n)))[:n:n]
}
func f64s(a *cArray, n int) []float64 {
	return (*[1 << 30]float64)(a.ensure(uintptr(n) * 8))[:n:n]
}

// nodeArrays / podArrays: the SoA inputs, in C memory, reused across calls.
type nodeArrays struct {
	cardNumber, freeSum, totalSum, alloc, free, total, clock, bw, core, power cArray
	cardCount, healthy, cpu, disk                                            cArray
}

type podArrays struct {
	hasNumber, hasMemory, hasClock, number, memory, clock, priority, rio, rcpu cArray
	pick, status                                                               cArray
}

// Handle owns one libyoda handle (one GPU, one node snapshot).  Not safe for concurrent
// use: the framework calls PreFilter once per pod cycle, cycles are serial.
type Handle struct {
	h         *C.yoda_t
	nodes     []string
	index     map[string]int
	zeroTotal []bool // Status.TotalMemorySum == 0 (the reference divides by it when scoring)
	na        nodeArrays
	pa        podArrays
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

// Close releases the device memory and the C-side arrays.
func (g *Handle) Close() {
	if g.h != nil {
		C.yoda_destroy(g.h)
		g.h = nil
	}
	g.na.release()
	for _, a := range []*cArray{&g.pa.hasNumber, &g.pa.hasMemory, &g.pa.hasClock, &g.pa.number,
		&g.pa.memory, &g.pa.clock, &g.pa.priority, &g.pa.rio, &g.pa.rcpu, &g.pa.pick,
		&g.pa.status} {
		a.free()
	}
}

// UploadNodes packs the SCV records (one per node, in the order of `names`) into the
// struct-of-arrays of yoda_node_soa and uploads them.  allocMemory[i] is the sum of the
// scv/memory labels of pods already on node i (score.CalculateAllocateScore's loop,
// algorithm.go:299-303); cpu/diskIO are advisor.NodeInfo values (Mode B, may be nil).
// scvs == nil: nodes without SCV records (Mode B, which reads none of them).
func (g *Handle) UploadNodes(names []string, scvs []*scv.Scv, allocMemory []uint64,
	cpu, diskIO []float64) error {
	return g.UploadShard(names, scvs, allocMemory, cpu, diskIO, 0)
}

// UploadShard is UploadNodes for one node shard of a multi-GPU snapshot: offset is the global
// index of names[0] (picks and node ids are global; see CommInit).  Shards exchange maxima, so
// they must agree on the record path and the N32 quotient type: exchange SmallFieldMax and
// RecordPath out of band and, when another shard's SmallFieldMax exceeds 55738, upload again
// with UploadShardFlags(..., UploadF64Quotients), then with UploadForceF64 where any shard
// reports PathF64 (include/yoda.h yoda_small_field_max; yoda_amd/dist.py agree_on_path).
func (g *Handle) UploadShard(names []string, scvs []*scv.Scv, allocMemory []uint64,
	cpu, diskIO []float64, offset uint32) error {
	return g.UploadShardFlags(names, scvs, allocMemory, cpu, diskIO, offset, 0)
}

// Upload flags (include/yoda.h YODA_UPLOAD_*) and record paths (YODA_PATH_*).
const (
	UploadForceF64     = uint32(C.YODA_UPLOAD_FORCE_F64)
	UploadF64Quotients = uint32(C.YODA_UPLOAD_F64_QUOTIENTS)
	PathN32            = int(C.YODA_PATH_N32)
	PathF64            = int(C.YODA_PATH_F64)
	PathU64            = int(C.YODA_PATH_U64)
)

// SmallFieldMax is the largest card bandwidth / clock / core / power of the uploaded snapshot.
func (g *Handle) SmallFieldMax() uint64 { return uint64(C.yoda_small_field_max(g.h)) }

// RecordPath is the uploaded snapshot's record format (PathN32, PathF64 or PathU64).
func (g *Handle) RecordPath() int { return int(C.yoda_record_path(g.h)) }

// UploadShardFlags is UploadShard with YODA_UPLOAD_* flags.
func (g *Handle) UploadShardFlags(names []string, scvs []*scv.Scv, allocMemory []uint64,
	cpu, diskIO []float64, offset uint32, flags uint32) error {
	n := len(names)
	if (scvs != nil && len(scvs) != n) || (allocMemory != nil && len(allocMemory) != n) {
		return errors.New("yodagpu: names/allocMemory do not match the SCV list")
	}
	if scvs == nil {
		scvs = make([]*scv.Scv, n)
		for i := range scvs {
			scvs[i] = &scv.Scv{}
		}
	}
	soa, zero, err := g.na.pack(scvs, allocMemory, cpu, diskIO)
	if err != nil {
		return err
	}
	// &soa is a Go pointer to memory holding only C pointers: allowed
	if err := check(g.h, C.yoda_upload_nodes(g.h, &soa, C.uint32_t(offset), C.uint32_t(flags)),
		"yoda_upload_nodes"); err != nil {
		return err
	}
	g.nodes = names
	g.zeroTotal = zero
	g.index = make(map[string]int, len(names))
	for i, name := range names {
		g.index[name] = i
	}
	return nil
}

// pack fills the C-side arrays of yoda_node_soa from the SCV records; zero[i]: node i has
// TotalMemorySum == 0.
func (a *nodeArrays) pack(scvs []*scv.Scv, allocMemory []uint64, cpu, diskIO []float64) (
	C.yoda_node_soa, []bool, error) {
	n := len(scvs)
	if (cpu == nil) != (diskIO == nil) || (cpu != nil && (len(cpu) != n || len(diskIO) != n)) {
		return C.yoda_node_soa{}, nil,
			errors.New("yodagpu: cpu/diskIO must both be nil or both have one value per node")
	}
	k := 1
	for _, s := range scvs {
		if len(s.Status.CardList) > k {
			k = len(s.Status.CardList)
		}
	}
	if k > C.YODA_MAX_CARDS {
		return C.yoda_node_soa{}, nil, errors.New("yodagpu: more than YODA_MAX_CARDS cards on a node")
	}
	cardNumber, cardCount := u64s(&a.cardNumber, n), u32s(&a.cardCount, n)
	freeSum, totalSum, alloc := u64s(&a.freeSum, n), u64s(&a.totalSum, n), u64s(&a.alloc, n)
	free, total, clock := u64s(&a.free, n*k), u64s(&a.total, n*k), u64s(&a.clock, n*k)
	bw, core, power := u64s(&a.bw, n*k), u64s(&a.core, n*k), u64s(&a.power, n*k)
	healthy := u8s(&a.healthy, n*k)
	zero := make([]bool, n)
	for i, s := range scvs {
		cardNumber[i] = uint64(s.Status.CardNumber)
		cardCount[i] = uint32(len(s.Status.CardList))
		freeSum[i] = s.Status.FreeMemorySum
		totalSum[i] = s.Status.TotalMemorySum
		zero[i] = s.Status.TotalMemorySum == 0
		alloc[i] = 0
		if allocMemory != nil {
			alloc[i] = allocMemory[i]
		}
		for j := 0; j < k; j++ {
			o := i*k + j
			free[o], total[o], clock[o], bw[o], core[o], power[o], healthy[o] = 0, 0, 0, 0, 0, 0, 0
		}
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
		card_number:      (*C.uint64_t)(a.cardNumber.p),
		card_count:       (*C.uint32_t)(a.cardCount.p),
		free_memory_sum:  (*C.uint64_t)(a.freeSum.p),
		total_memory_sum: (*C.uint64_t)(a.totalSum.p),
		alloc_memory:     (*C.uint64_t)(a.alloc.p),
		card_free_memory: (*C.uint64_t)(a.free.p), card_total_memory: (*C.uint64_t)(a.total.p),
		card_clock: (*C.uint64_t)(a.clock.p), card_bandwidth: (*C.uint64_t)(a.bw.p),
		card_core: (*C.uint64_t)(a.core.p), card_power: (*C.uint64_t)(a.power.p),
		card_healthy: (*C.uint8_t)(a.healthy.p),
	}
	if cpu != nil {
		copy(f64s(&a.cpu, n), cpu)
		copy(f64s(&a.disk, n), diskIO)
		soa.cpu = (*C.double)(a.cpu.p)
		soa.disk_io = (*C.double)(a.disk.p)
	}
	return soa, zero, nil
}

func (a *nodeArrays) release() {
	for _, x := range []*cArray{&a.cardNumber, &a.freeSum, &a.totalSum, &a.alloc, &a.free,
		&a.total, &a.clock, &a.bw, &a.core, &a.power, &a.cardCount, &a.healthy, &a.cpu, &a.disk} {
		x.free()
	}
}

// SetNodeState updates the allocated scv/memory (and CardNumber) of a few nodes on the
// device without re-uploading the snapshot (yoda_set_node_state): the scheduler's assumes
// and binds between two cycles.  idx are snapshot positions.
func (g *Handle) SetNodeState(idx []uint32, alloc, cardNumber []uint64) error {
	if len(idx) != len(alloc) || len(idx) != len(cardNumber) {
		return errors.New("yodagpu: SetNodeState arrays differ in length")
	}
	if len(idx) == 0 {
		return nil
	}
	// plain-number Go slices passed directly as arguments: allowed by the cgo rules
	rc := C.yoda_set_node_state(g.h, C.uint32_t(len(idx)), (*C.uint32_t)(unsafe.Pointer(&idx[0])),
		(*C.uint64_t)(unsafe.Pointer(&alloc[0])), (*C.uint64_t)(unsafe.Pointer(&cardNumber[0])))
	return check(g.h, rc, "yoda_set_node_state")
}

// packPods parses the scv/* labels and the diskIO annotation with the reference's own
// helpers (filter.go:60-74, sort.go:12-18, algorithm.go:103-104) into the C-side
// yoda_pod_soa arrays.
func (g *Handle) packPods(pods []*v1.Pod) C.yoda_pod_soa {
	n := len(pods)
	a := &g.pa
	hasNumber, hasMemory, hasClock := u8s(&a.hasNumber, n), u8s(&a.hasMemory, n), u8s(&a.hasClock, n)
	number, memory, clock := u64s(&a.number, n), u64s(&a.memory, n), u64s(&a.clock, n)
	priority, rcpu, rio := i64s(&a.priority, n), i64s(&a.rcpu, n), f64s(&a.rio, n)
	for i, p := range pods {
		l := p.GetLabels()
		has := func(key string) (uint8, uint64) {
			if v, ok := l[key]; ok {
				return 1, filter.StrToUint64(v)
			}
			return 0, 0
		}
		hasNumber[i], number[i] = has("scv/number")
		hasMemory[i], memory[i] = has("scv/memory")
		hasClock[i], clock[i] = has("scv/clock")
		priority[i] = 0
		if v, ok := l["scv/priority"]; ok {
			pr, _ := strconv.Atoi(v) // sort.go:14-15 keeps Atoi's value on error
			priority[i] = int64(pr)
		}
		rio[i], _ = strconv.ParseFloat(p.Annotations["diskIO"], 32) // algorithm.go:103
		rcpu[i] = score.CalculatePodResourceRequest(p, v1.ResourceCPU, true)
	}
	return C.yoda_pod_soa{
		n_pods:     C.uint32_t(n),
		has_number: (*C.uint8_t)(a.hasNumber.p), number: (*C.uint64_t)(a.number.p),
		has_memory: (*C.uint8_t)(a.hasMemory.p), memory: (*C.uint64_t)(a.memory.p),
		has_clock: (*C.uint8_t)(a.hasClock.p), clock: (*C.uint64_t)(a.clock.p),
		priority: (*C.int64_t)(a.priority.p), rio: (*C.double)(a.rio.p),
		rcpu: (*C.int64_t)(a.rcpu.p),
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
	s := g.packPods([]*v1.Pod{pod})
	if err := check(g.h, C.yoda_upload_pods(g.h, &s), "yoda_upload_pods"); err != nil {
		return nil, err
	}
	n := len(g.nodes)
	row := &Row{Feasible: make([]uint32, (n+31)/32+1), Score: make([]int64, n+1)}
	rc := C.yoda_score_rows(g.h, C.int(mode), (*C.uint32_t)(unsafe.Pointer(&row.Feasible[0])),
		C.uint64_t((n+31)/32), (*C.int64_t)(unsafe.Pointer(&row.Score[0])), C.uint64_t(n))
	if err := check(g.h, rc, "yoda_score_rows"); err != nil {
		return nil, err
	}
	row.Feasible, row.Score = row.Feasible[:(n+31)/32], row.Score[:n]
	return row, nil
}

// Batch schedules many pods independently against the snapshot (configs 2-4).  Picks are
// node indices, -1 unschedulable, -2 error (see statuses).
func (g *Handle) Batch(pods []*v1.Pod, mode Mode) (picks []int32, statuses []int32, err error) {
	if len(pods) == 0 {
		return nil, nil, nil
	}
	s := g.packPods(pods)
	n := len(pods)
	pk, st := i32s(&g.pa.pick, n), i32s(&g.pa.status, n)
	out := C.yoda_eval_out{pick: (*C.int32_t)(g.pa.pick.p), status: (*C.int32_t)(g.pa.status.p)}
	if err = check(g.h, C.yoda_eval(g.h, &s, C.int(mode), &out), "yoda_eval"); err != nil {
		return nil, nil, err
	}
	return append([]int32(nil), pk...), append([]int32(nil), st...), nil
}

// Greedy schedules the pods one after another in sort.Less order, each pick updating the
// node's Allocate score (config 5); cardCapacity also decrements CardNumber.
func (g *Handle) Greedy(pods []*v1.Pod, mode Mode, cardCapacity bool) ([]int32, error) {
	if len(pods) == 0 {
		return nil, nil
	}
	s := g.packPods(pods)
	picks := make([]int32, len(pods))
	flags := C.uint32_t(0)
	if cardCapacity {
		flags = C.YODA_GREEDY_CARD_CAPACITY
	}
	rc := C.yoda_greedy(g.h, &s, C.int(mode), flags, (*C.int32_t)(unsafe.Pointer(&picks[0])))
	return picks, check(g.h, rc, "yoda_greedy")
}

// ---- several GPUs: libyoda's own RCCL exchange (include/yoda.h yoda_comm_*) --------------

// CommUniqueID makes the communicator id on rank 0; hand it to the other ranks out of band
// (a file, a ConfigMap, the k8s API ...).
func CommUniqueID() ([]byte, error) {
	id := make([]byte, C.YODA_COMM_ID_BYTES)
	if err := check(nil, C.yoda_comm_unique_id((*C.uint8_t)(unsafe.Pointer(&id[0]))),
		"yoda_comm_unique_id"); err != nil {
		return nil, err
	}
	return id, nil
}

// DeviceKey identifies this handle's GPU across hosts (yoda_device_key: a hash of the hostname
// and boot id, '/', the PCI bus id -- bus ids alone repeat on identical servers).  Ranks
// exchange it with the communicator id, out of band, and call CheckDevices before CommInit.
func (g *Handle) DeviceKey() (string, error) {
	buf := make([]byte, C.YODA_DEVICE_KEY_BYTES)
	if err := check(g.h, C.yoda_device_key(g.h, (*C.char)(unsafe.Pointer(&buf[0])),
		C.int(len(buf))), "yoda_device_key"); err != nil {
		return "", err
	}
	return C.GoString((*C.char)(unsafe.Pointer(&buf[0]))), nil
}

// DeviceBusID is the PCI bus id of this handle's GPU (yoda_device_bus_id).
func (g *Handle) DeviceBusID() (string, error) {
	buf := make([]byte, C.YODA_BUS_ID_BYTES)
	if err := check(g.h, C.yoda_device_bus_id(g.h, (*C.char)(unsafe.Pointer(&buf[0])),
		C.int(len(buf))), "yoda_device_bus_id"); err != nil {
		return "", err
	}
	return C.GoString((*C.char)(unsafe.Pointer(&buf[0]))), nil
}

// CheckDevices takes every rank's DeviceKey (rank order) and fails, naming the first pair,
// when two ranks would share one GPU (YODA_ERR_SAME_DEVICE: RCCL itself only reports an
// "invalid usage").  Host only.
func CheckDevices(busIDs []string) error {
	if len(busIDs) == 0 {
		return nil
	}
	stride := int(C.YODA_DEVICE_KEY_BYTES)
	flat := make([]byte, stride*len(busIDs))
	for r, id := range busIDs {
		if len(id) >= stride {
			return fmt.Errorf("yodagpu: device key of rank %d too long", r)
		}
		copy(flat[r*stride:], id)
	}
	var a, b C.int
	rc := C.yoda_comm_check_devices((*C.char)(unsafe.Pointer(&flat[0])), C.int(len(busIDs)),
		C.int(stride), &a, &b)
	if rc == C.YODA_ERR_SAME_DEVICE {
		return fmt.Errorf("yodagpu: ranks %d and %d are on the same GPU (%s)", int(a), int(b),
			busIDs[a])
	}
	return check(nil, rc, "yoda_comm_check_devices")
}

// CommInit joins this handle (one GPU holding the node shard uploaded with UploadShard) to the
// communicator of `world` ranks; collective: every rank calls it.
func (g *Handle) CommInit(id []byte, rank, world int) error {
	if len(id) != C.YODA_COMM_ID_BYTES {
		return errors.New("yodagpu: communicator id of the wrong size")
	}
	return check(g.h, C.yoda_comm_init(g.h, (*C.uint8_t)(unsafe.Pointer(&id[0])), C.int(rank),
		C.int(world)), "yoda_comm_init")
}

// ShardedBatch schedules the pods against the node shards of every rank (collective: every
// rank passes the same pods): yoda_comm_run's maxima / packed-key all-reduces.  Picks are
// global node indices.
func (g *Handle) ShardedBatch(pods []*v1.Pod, mode Mode) (picks []int32, statuses []int32, err error) {
	if len(pods) == 0 {
		return nil, nil, nil
	}
	s := g.packPods(pods)
	n := len(pods)
	if err = check(g.h, C.yoda_upload_pods(g.h, &s), "yoda_upload_pods"); err != nil {
		return nil, nil, err
	}
	if err = check(g.h, C.yoda_comm_run(g.h, C.int(mode)), "yoda_comm_run"); err != nil {
		return nil, nil, err
	}
	pk, st := i32s(&g.pa.pick, n), i32s(&g.pa.status, n)
	out := C.yoda_eval_out{pick: (*C.int32_t)(g.pa.pick.p), status: (*C.int32_t)(g.pa.status.p)}
	if err = check(g.h, C.yoda_download(g.h, &out), "yoda_download"); err != nil {
		return nil, nil, err
	}
	return append([]int32(nil), pk...), append([]int32(nil), st...), nil
}

// ShardedGreedy is Greedy across the ranks' node shards (collective; every rank passes the
// same pods and the same full snapshot `all`, which the host-side resolve reads): the windows'
// maxima and candidate lists merged over RCCL inside libyoda (yoda_comm_greedy).
func (g *Handle) ShardedGreedy(all []*scv.Scv, allAlloc []uint64, pods []*v1.Pod, mode Mode,
	cardCapacity bool) ([]int32, error) {
	if len(pods) == 0 {
		return nil, nil
	}
	var full nodeArrays // the full snapshot's C arrays (host only)
	defer full.release()
	soa, _, err := full.pack(all, allAlloc, nil, nil)
	if err != nil {
		return nil, err
	}
	s := g.packPods(pods)
	picks := make([]int32, len(pods))
	flags := C.uint32_t(0)
	if cardCapacity {
		flags = C.YODA_GREEDY_CARD_CAPACITY
	}
	rc := C.yoda_comm_greedy(g.h, &soa, &s, C.int(mode), flags,
		(*C.int32_t)(unsafe.Pointer(&picks[0])))
	return picks, check(g.h, rc, "yoda_comm_greedy")
}

// NodeIndex maps a node name to its row position.
func (g *Handle) NodeIndex(name string) (int, bool) {
	i, ok := g.index[name]
	return i, ok
}

// ZeroTotal reports whether node i has TotalMemorySum == 0: scoring it divides by zero in
// the reference (algorithm.go:294,309), a framework Error here.
func (g *Handle) ZeroTotal(i int) bool { return i >= 0 && i < len(g.zeroTotal) && g.zeroTotal[i] }

// Nodes is the snapshot's node order.
func (g *Handle) Nodes() []string { return g.nodes }
