package gwaoi

/*
#include "gwaoi_strips.h"
*/
import "C"

import "unsafe"

// StripComm is the RCCL communicator of one X-strip world (include/gwaoi_strips.h, SURVEY 8(e)
// config 4): one game process per GPU, each owning the entities whose x lies in its strip.
type StripComm struct{ c *C.gwaoi_strip_comm }

// NewStripCommID makes the 128-byte id on rank 0; the deployment's own transport hands it to the other
// ranks (the dispatcher, or a file on shared storage).
func NewStripCommID() []byte {
	id := make([]byte, C.GWAOI_STRIP_COMM_ID_BYTES)
	chk(C.gwaoi_strip_comm_id((*C.uint8_t)(unsafe.Pointer(&id[0]))))
	return id
}

func NewStripComm(id []byte, nRanks, rank, device int) *StripComm {
	s := &StripComm{}
	chk(C.gwaoi_strip_comm_init((*C.uint8_t)(unsafe.Pointer(&id[0])), C.int(nRanks), C.int(rank), C.int(device), &s.c))
	return s
}

func (s *StripComm) Close() {
	if s.c != nil {
		C.gwaoi_strip_comm_destroy(s.c)
		s.c = nil
	}
}

// StripTick is one rank's tick (goworld_amd/strips.py StripNode.tick_rccl is the tested host of the same
// sequence). All buffers are device memory sized at set-up (d.* below); every call enqueues on `stream`
// and nothing waits on the host before the manager's own end-of-pass read.
type StripDev struct {
	Stream                          unsafe.Pointer // hipStream_t the manager also uses (gwaoi_set_stream)
	Geom                            C.gwaoi_strip_geom
	Flags                           *C.uint8_t
	SX, SZ, EX, EZ                  *C.float
	Left, Right, LeftIn, RightIn    *C.uint32_t // haloCap records of 4 x uint32
	Counts, CountsIn, Err           *C.uint32_t
	HaloCap                         uint32
	OpSlots                         *C.uint32_t
	OpX, OpZ                        *C.float
	OpKinds                         *C.uint8_t
	Scratch, NOps                   *C.uint32_t
	G2L, L2G, FreeQ, Pend, LocalCtr *C.uint32_t
	CapL                            uint32
	Bound                           uint32 // op bound for gwaoi_stage_ops_device_n
}

func (g *Manager) StripTick(comm *StripComm, d *StripDev, left, right int, ids *C.uint32_t, xs, zs *C.float, nMoves uint32) {
	st := d.Stream
	chk(C.gwaoi_strip_ingest(st, &d.Geom, d.Flags, d.SX, d.EX, d.EZ, ids, xs, zs, C.uint32_t(nMoves), d.Err))
	chk(C.gwaoi_strip_select(st, &d.Geom, d.Flags, d.SX, d.EX, d.EZ, d.Left, d.Right, C.uint32_t(d.HaloCap), d.Counts, d.Err))
	chk(C.gwaoi_strip_exchange(comm.c, st, C.int(left), C.int(right), d.Left, d.Right, d.Counts, C.uint32_t(d.HaloCap),
		d.LeftIn, d.RightIn, d.CountsIn))
	in := unsafe.Slice(d.CountsIn, 2)
	if left >= 0 {
		chk(C.gwaoi_strip_absorb_n(st, d.Flags, d.EX, d.EZ, d.LeftIn, &in[0], C.uint32_t(d.HaloCap), d.Err))
	}
	if right >= 0 {
		chk(C.gwaoi_strip_absorb_n(st, d.Flags, d.EX, d.EZ, d.RightIn, &in[1], C.uint32_t(d.HaloCap), d.Err))
	}
	chk(C.gwaoi_strip_emit_local(st, &d.Geom, d.Flags, d.SX, d.SZ, d.EX, d.EZ, d.OpSlots, d.OpX, d.OpZ, d.OpKinds,
		d.Scratch, d.NOps, d.G2L, d.L2G, d.FreeQ, d.Pend, C.uint32_t(d.CapL), d.LocalCtr))
	chk(C.gwaoi_stage_ops_device_n(g.m, d.OpSlots, d.OpX, d.OpZ, d.OpKinds, nil, d.NOps, C.uint32_t(d.Bound)))
	// then Flush: the events of this rank's owned movers (local slots: translate with
	// gwaoi_strip_translate_events before the replay), and read d.Err / LocalCtr[3] for protocol errors
}

// StripRegionDev is the same rank's tick on a region state (ABI 2.1, include/gwaoi_strips.h: the strip's state in
// the manager's local-slot order, so the per-tick kernels follow the region's population, not the world's id
// range). Region holds the device buffers (allocated at set-up, gwaoi_strip_region_init, then tick 0 by
// gwaoi_strip_region_start); the emit flips Region.cur, so the struct is passed by pointer every tick.
type StripRegionDev struct {
	Stream                       unsafe.Pointer
	Geom                         C.gwaoi_strip_geom
	Region                       C.gwaoi_strip_region
	Left, Right, LeftIn, RightIn *C.uint32_t
	Counts, CountsIn, Err        *C.uint32_t
	HaloCap                      uint32
	OpSlots                      *C.uint32_t
	OpX, OpZ                     *C.float
	OpKinds                      *C.uint8_t
	NOps                         *C.uint32_t
	Bound                        uint32
}

func (g *Manager) StripTickRegion(comm *StripComm, d *StripRegionDev, left, right int, ids *C.uint32_t, xs, zs *C.float,
	nMoves uint32) {
	st := d.Stream
	chk(C.gwaoi_strip_region_ingest(st, &d.Geom, &d.Region, ids, xs, zs, C.uint32_t(nMoves), d.Err))
	if left < 0 && right < 0 { // a one-strip world: nothing to select or exchange
		chk(C.gwaoi_strip_region_emit(st, &d.Geom, &d.Region, d.OpSlots, d.OpX, d.OpZ, d.OpKinds, d.NOps))
		chk(C.gwaoi_stage_ops_device_n(g.m, d.OpSlots, d.OpX, d.OpZ, d.OpKinds, nil, d.NOps, C.uint32_t(d.Bound)))
		return
	}
	chk(C.gwaoi_strip_region_select(st, &d.Geom, &d.Region, d.Left, d.Right, C.uint32_t(d.HaloCap), d.Counts, d.Err))
	chk(C.gwaoi_strip_exchange(comm.c, st, C.int(left), C.int(right), d.Left, d.Right, d.Counts, C.uint32_t(d.HaloCap),
		d.LeftIn, d.RightIn, d.CountsIn))
	in := unsafe.Slice(d.CountsIn, 2)
	var nl, nr C.uint32_t
	var dl, dr *C.uint32_t
	if left >= 0 {
		nl, dl = C.uint32_t(d.HaloCap), &in[0]
	}
	if right >= 0 {
		nr, dr = C.uint32_t(d.HaloCap), &in[1]
	}
	chk(C.gwaoi_strip_region_absorb2(st, &d.Region, d.LeftIn, dl, nl, d.RightIn, dr, nr, d.Err))
	chk(C.gwaoi_strip_region_emit(st, &d.Geom, &d.Region, d.OpSlots, d.OpX, d.OpZ, d.OpKinds, d.NOps))
	chk(C.gwaoi_stage_ops_device_n(g.m, d.OpSlots, d.OpX, d.OpZ, d.OpKinds, nil, d.NOps, C.uint32_t(d.Bound)))
	// then Flush, translate the events with Region.l2g (gwaoi_strip_translate_events), and read d.Err,
	// Region.lctr[3] and Region.ctr[6] for protocol errors
}
