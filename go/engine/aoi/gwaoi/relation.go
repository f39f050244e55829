package gwaoi

/*
#include "gwaoi.h"
*/
import "C"

import (
	"sort"

	"github.com/xiaonanln/go-aoi"
	"github.com/xiaonanln/goworld/engine/gwlog"
)

// Sets keeps every entity's neighbour set (InterestedIn == InterestedBy under the XZ manager,
// Entity.go:53-54) as a sorted slot slice, patched once per tick with the relation's net changes
// (gwaoi_export_relation_delta: O(events) on the GPU and over PCIe) instead of re-exporting the whole
// relation or replaying every event into maps. Readers: CollectEntitySyncInfos' InterestedBy loop
// (Entity.go:1241), examples/unity_demo/Monster.go:50,79,89 (InterestedIn).
type Sets struct {
	rows   [][]uint32
	buf    []C.gwaoi_event
	bySlot []*aoi.AOI
}

// Load copies the current relation once (gwaoi_export_relation), e.g. after a restore.
func (g *Manager) Load(s *Sets) {
	if g.nmv > 0 {
		gwlog.Panicf("gwaoi: Load with moves pending; Flush first")
	}
	rowPtr := make([]uint32, len(g.bySlot)+1)
	cols := make([]uint32, 1024)
	var nnz C.uint64_t
	rc := C.gwaoi_export_relation(g.m, (*C.uint32_t)(&rowPtr[0]), (*C.uint32_t)(&cols[0]), C.uint64_t(len(cols)), &nnz)
	if rc == C.GWAOI_ERR_INVALID && uint64(nnz) > uint64(len(cols)) {
		cols = make([]uint32, nnz)
		rc = C.gwaoi_export_relation(g.m, (*C.uint32_t)(&rowPtr[0]), (*C.uint32_t)(&cols[0]), C.uint64_t(len(cols)), &nnz)
	}
	chk(rc)
	s.rows = make([][]uint32, len(g.bySlot))
	for r := range s.rows {
		s.rows[r] = append([]uint32(nil), cols[rowPtr[r]:rowPtr[r+1]]...)
	}
	s.bySlot = g.bySlot
}

// ApplyDelta patches the sets with the last Flush's net changes. Call it after Flush and before the
// next Enter/Leave/Moved push (the library refuses it once another pass ran).
func (g *Manager) ApplyDelta(s *Sets) {
	if len(s.buf) == 0 {
		s.buf = make([]C.gwaoi_event, 1<<16)
	}
	var n C.uint64_t
	rc := C.gwaoi_export_relation_delta(g.m, &s.buf[0], C.uint64_t(len(s.buf)), &n)
	if rc == C.GWAOI_ERR_INVALID && uint64(n) > uint64(len(s.buf)) {
		s.buf = make([]C.gwaoi_event, n+n/4)
		rc = C.gwaoi_export_relation_delta(g.m, &s.buf[0], C.uint64_t(len(s.buf)), &n)
	}
	chk(rc)
	for _, e := range s.buf[:n] {
		row, col := uint32(e.mover), uint32(e.other&C.GWAOI_EV_SLOT_MASK)
		a := s.rows[row]
		p := sort.Search(len(a), func(i int) bool { return a[i] >= col })
		if e.other&C.GWAOI_EV_ENTER != 0 {
			a = append(a, 0)
			copy(a[p+1:], a[p:])
			a[p] = col
		} else {
			a = append(a[:p], a[p+1:]...)
		}
		s.rows[row] = a
	}
	s.bySlot = g.bySlot
}

// InterestedBy calls f for every entity whose AOI contains slot a (Entity.go:1241's loop).
func (s *Sets) InterestedBy(a uint32, f func(other *aoi.AOI)) {
	for _, o := range s.rows[a] {
		f(s.bySlot[o])
	}
}
