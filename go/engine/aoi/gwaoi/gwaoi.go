// Package gwaoi is a GPU-backed aoi.AOIManager for GoWorld: libgwaoi (hand-written HIP for AMD
// MI355X / gfx950) behind go-aoi's AOIManager interface, which engine/entity's Space already holds
// (engine/entity/Space.go:33). It replaces aoi.NewXZListAOIManager (Space.go:105); Space.enter,
// Space.leave and Space.move (Space.go:211,221,243,259) are unchanged.
//
// Place this directory at engine/aoi/gwaoi of the goworld tree, libgwaoi.so and include/ at gwaoi/
// (see Makefile.gwaoi). Written against include/gwaoi.h ABI 2; not compiled in the repository that
// holds it (no Go toolchain there): tests/abi_smoke.c drives the same C calls in the same order from
// plain C, and goworld_amd/aoi.py is the same wrapper over ctypes, both tested on the GPU.
package gwaoi

/*
#cgo CFLAGS: -I${SRCDIR}/../../../gwaoi/include
#cgo LDFLAGS: -L${SRCDIR}/../../../gwaoi/lib -lgwaoi -Wl,-rpath,${SRCDIR}/../../../gwaoi/lib
#include <stdlib.h>
#include "gwaoi.h"
*/
import "C"

import (
	"unsafe"

	"github.com/xiaonanln/go-aoi"
	"github.com/xiaonanln/goworld/engine/gwlog"
)

// Manager satisfies aoi.AOIManager. Moved writes the call into the manager's pinned staging arrays
// (library-owned C memory, so no cgo crossing and no copy); the pending moves reach the GPU in ONE
// gwaoi_stage_moves_pinned call before the next Enter/Leave (which must stay ordered after them) or at
// Flush, validated there. Flush (once per game tick) runs the GPU pipeline and replays the events into
// the callbacks in canonical order.
type Manager struct {
	m        *C.gwaoi_mgr
	bySlot   []*aoi.AOI
	slotOf   map[*aoi.AOI]uint32
	free     []uint32
	released []uint32
	// pending Moved calls in call order, in pinned C memory (a slot may repeat: the library splits the
	// batch into sub-passes where it does, so every call keeps its sequential meaning)
	pinSlot []uint32
	pinX    []float32
	pinZ    []float32
	nmv     int
	pushed  int // pending calls already copied to the device (gwaoi_stage_moves_pinned_partial)
	// PushEvery > 0: every PushEvery Moved calls the filled part of the staging arrays is copied to the
	// device while the tick goes on (ABI 2.1), so Flush copies only the tail
	PushEvery int
	// SyncEnterLeave flushes inside Enter/Leave so their callbacks fire before Space.enter runs the
	// user hooks (Space.go:211-217), exactly as with the list manager.
	SyncEnterLeave bool
}

func chk(rc C.int) {
	if rc != C.GWAOI_OK {
		gwlog.Panicf("gwaoi: %d: %s", int(rc), C.GoString(C.gwaoi_last_error()))
	}
}

// NewXZListAOIManager has the signature of go-aoi's constructor (Space.go:105) plus capacity/device.
func NewXZListAOIManager(aoidist aoi.Coord, capacity uint32, device int) *Manager {
	if v := int(C.gwaoi_abi_version()); v != int(C.GWAOI_ABI_VERSION) {
		gwlog.Panicf("gwaoi: libgwaoi.so has ABI %d, these headers %d", v, int(C.GWAOI_ABI_VERSION))
	}
	if int(C.gwaoi_abi_minor()) < 1 {
		gwlog.Panicf("gwaoi: libgwaoi.so predates ABI 2.1 (gwaoi_stage_moves_pinned_async / _partial)")
	}
	g := &Manager{bySlot: make([]*aoi.AOI, capacity), slotOf: map[*aoi.AOI]uint32{}, SyncEnterLeave: true,
		PushEvery: 65536}
	for s := int(capacity) - 1; s >= 0; s-- {
		g.free = append(g.free, uint32(s))
	}
	chk(C.gwaoi_create(C.float(aoidist), C.uint32_t(capacity), C.int(device), &g.m))
	var ps *C.uint32_t
	var px, pz *C.float
	var n C.uint32_t
	chk(C.gwaoi_stage_buffers(g.m, &ps, &px, &pz, &n))
	// Go may keep pointers into C memory: the arrays belong to the manager until Close
	g.pinSlot = unsafe.Slice((*uint32)(unsafe.Pointer(ps)), int(n))
	g.pinX = unsafe.Slice((*float32)(unsafe.Pointer(px)), int(n))
	g.pinZ = unsafe.Slice((*float32)(unsafe.Pointer(pz)), int(n))
	return g
}

// pushMoves hands the pending Moved calls to the manager: one cgo crossing, one DMA copy of what was not
// pushed yet. The device checks the batch and its verdict is read by the pass that runs it
// (gwaoi_stage_moves_pinned_async): a refused batch panics at the next gwaoi_tick, with nothing of it
// applied, as it would have here.
func (g *Manager) pushMoves() {
	if g.nmv > 0 {
		n := g.nmv
		g.nmv, g.pushed = 0, 0
		chk(C.gwaoi_stage_moves_pinned_async(g.m, C.uint32_t(n)))
	}
}

func (g *Manager) Enter(a *aoi.AOI, x, y aoi.Coord) {
	g.pushMoves() // ops apply in call order
	if len(g.free) == 0 {
		gwlog.Panicf("gwaoi: manager capacity %d exhausted", len(g.bySlot))
	}
	slot := g.free[len(g.free)-1]
	g.free = g.free[:len(g.free)-1]
	g.bySlot[slot], g.slotOf[a] = a, slot
	chk(C.gwaoi_enter(g.m, C.uint32_t(slot), C.float(x), C.float(y)))
	if g.SyncEnterLeave {
		g.Flush()
	}
}

func (g *Manager) Leave(a *aoi.AOI) {
	g.pushMoves()
	slot, ok := g.slotOf[a]
	if !ok {
		gwlog.Panicf("gwaoi: Leave of an AOI that is not in the manager")
	}
	delete(g.slotOf, a)
	chk(C.gwaoi_leave(g.m, C.uint32_t(slot)))
	g.released = append(g.released, slot) // reusable once its events are replayed
	if g.SyncEnterLeave {
		g.Flush()
	}
}

// Moved: no cgo call. A Moved of an AOI that is not in the manager panics here (the reference's list
// manager would corrupt its lists); the library re-checks every slot on the GPU when the batch is
// pushed and refuses non-finite coordinates (GWAOI_ERR_INVALID, nothing of the batch staged).
func (g *Manager) Moved(a *aoi.AOI, x, y aoi.Coord) {
	slot, ok := g.slotOf[a]
	if !ok {
		gwlog.Panicf("gwaoi: Moved of an AOI that is not in the manager")
	}
	k := g.nmv
	g.pinSlot[k], g.pinX[k], g.pinZ[k] = slot, float32(x), float32(y)
	g.nmv = k + 1
	if g.nmv == len(g.pinSlot) {
		g.pushMoves()
	} else if g.PushEvery > 0 && g.nmv-g.pushed >= g.PushEvery {
		// the filled part travels now (asynchronous DMA, nothing staged yet): Flush copies only the tail
		chk(C.gwaoi_stage_moves_pinned_partial(g.m, C.uint32_t(g.nmv)))
		g.pushed = g.nmv
	}
}

// Flush applies every staged call and fires the callbacks, mover's first
// (aoi.callback.OnEnterAOI(other) then other.callback.OnEnterAOI(aoi), as go-aoi does).
func (g *Manager) Flush() {
	g.pushMoves()
	var ev C.gwaoi_events
	chk(C.gwaoi_tick(g.m, &ev))
	events := unsafe.Slice((*C.gwaoi_event)(unsafe.Pointer(ev.events)), int(ev.count))
	for _, e := range events {
		a := g.bySlot[e.mover]
		o := g.bySlot[e.other&C.GWAOI_EV_SLOT_MASK]
		// go-aoi's AOI.callback is unexported; GoWorld passes the *Entity as both Data and callback
		// (Entity.go:210: aoi.InitAOI(&e.aoi, dist, e, e)), so the callback is reachable through Data.
		ca, co := a.Data.(aoi.AOICallback), o.Data.(aoi.AOICallback)
		if e.other&C.GWAOI_EV_ENTER != 0 {
			ca.OnEnterAOI(o)
			co.OnEnterAOI(a)
		} else {
			ca.OnLeaveAOI(o)
			co.OnLeaveAOI(a)
		}
	}
	for _, s := range g.released {
		g.bySlot[s] = nil
		g.free = append(g.free, s)
	}
	g.released = g.released[:0]
}

// Close releases the manager and its device memory; the staging slices die with it.
func (g *Manager) Close() {
	g.pinSlot, g.pinX, g.pinZ = nil, nil, nil
	if g.m != nil {
		C.gwaoi_destroy(g.m)
		g.m = nil
	}
}
