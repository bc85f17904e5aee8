//go:build mirsha
// +build mirsha

// GPU-batched SHA-256 for MirBFT's hash path, backed by libmirsha (the C ABI in
// include/mirsha.h of the mirbft_amd repository).
//
// This file belongs in the reference tree at pkg/processor/gpuhash.go (package
// processor); go/wiring.patch adds the three call sites that use it. It replaces,
// for a whole batch at a time:
//
//   - ProcessHashActions (pkg/processor/serial.go:180-198): ProcessHashActionsGPU
//     has the same arguments, the same result order, the same Origin pointers and
//     the same error for a non-hash action, but makes ONE libmirsha call per
//     ActionList instead of one hash.Hash per action;
//   - the request digest of Client.Propose (pkg/processor/clients.go:189-192):
//     Client.ProposeBatch hashes several requests in one call, then runs
//     Propose's own bookkeeping (proposeDigest, split out of Propose by the
//     patch) for each request in order.
//
// The per-message processor.Hasher (crypto.SHA256) stays what the node uses for
// single Propose calls and the testengine's application hash chain; libmirsha
// has no CPU fallback of its own.
//
// cgo rules followed here: Go memory passed to C holds no Go pointers (the
// [][]byte parts are packed into one arena first), and the arena and digest
// buffers are page-locked C memory from msha_pinned_alloc, so the library DMAs
// them as is. Digests are copied into fresh Go slices: the state machine keeps
// them as map keys (batch_tracker.go:85-91, epoch_change.go:42-50).
//
// Built only with the mirsha build tag (go build -tags mirsha), because it links
// libmirsha through cgo. Without the tag gpuhash_stub.go declares the same API
// with no cgo and no library, so the reference's CI (ginkgo -r, staticcheck
// ./..., CGO_ENABLED=0) builds the patched tree unchanged; gpuhash_api.go holds
// what both builds share. tests/test_go_adapter.py (mirbft_amd repository)
// checks that the two files declare the same exported API.
//
// Go 1.15 compatible (go.mod:3): no generics, no unsafe.Slice.
package processor

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/mirsha/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/mirsha/lib -lmirsha -Wl,-rpath,${SRCDIR}/../../third_party/mirsha/lib
#include <stdlib.h>
#include "mirsha.h"
*/
import "C"

import (
	"sync"
	"unsafe"

	"github.com/pkg/errors"

	"github.com/hyperledger-labs/mirbft/pkg/pb/msgs"
	"github.com/hyperledger-labs/mirbft/pkg/pb/state"
	"github.com/hyperledger-labs/mirbft/pkg/statemachine"
)

// GPUHasher owns one libmirsha context (on the GPUs of its device mask) and two
// pinned buffers: the packing arena and the digest output. libmirsha serialises
// calls on a shared context (mirsha.h), but the pinned buffers and the packing
// slices here are per GPUHasher, so the mutex makes every call exclusive: the
// hash goroutine (mirbft.go:470) and ProposeBatch callers can share one
// GPUHasher, and msha_last_error(ctx) is read before any other call can start.
type GPUHasher struct {
	mutex  sync.Mutex
	ctx    *C.msha_ctx
	arena  pinnedBuf
	out    pinnedBuf
	off    pinnedBuf // uint64 per message
	length pinnedBuf // uint64 per message
}

type pinnedBuf struct {
	base unsafe.Pointer
	buf  []byte
}

// NewGPUHasher creates a libmirsha context over the GPUs in deviceMask (bit i
// = HIP device i; 0 means device 0). Independent hash actions are sharded over
// them by cumulative block count; there is no collective.
func NewGPUHasher(deviceMask uint32) (*GPUHasher, error) {
	var ctx *C.msha_ctx
	var errbuf [512]C.char
	// The creation error travels with the call (msha_ctx_create_err): a
	// goroutine may resume on another OS thread between two cgo calls.
	rc := C.msha_ctx_create_err(C.uint32_t(deviceMask), &ctx, &errbuf[0], C.uint64_t(len(errbuf)))
	if rc != C.MSHA_OK {
		return nil, errors.Errorf("libmirsha error %d: %s", int(rc), C.GoString(&errbuf[0]))
	}
	return &GPUHasher{ctx: ctx}, nil
}

// Close releases the pinned buffers and the context.
func (g *GPUHasher) Close() {
	g.mutex.Lock()
	defer g.mutex.Unlock()
	if g.ctx == nil {
		return
	}
	for _, p := range []*pinnedBuf{&g.arena, &g.out, &g.off, &g.length} {
		if p.base != nil {
			C.msha_pinned_free(g.ctx, p.base)
			p.base, p.buf = nil, nil
		}
	}
	C.msha_ctx_destroy(g.ctx)
	g.ctx = nil
}

func (g *GPUHasher) fail(rc C.int) error {
	// The context is used under g.mutex only, so the text belongs to this call
	// whatever thread reads it; msha_last_error_copy also reads it under the
	// library's own lock.
	var buf [512]C.char
	C.msha_last_error_copy(g.ctx, &buf[0], C.uint64_t(len(buf)))
	return errors.Errorf("libmirsha error %d: %s", int(rc), C.GoString(&buf[0]))
}

// lastPayloadUpload is the payload bytes the last call uploaded, summed over
// the context's GPUs (msha_get_shard_stats.h2d_payload_bytes; for tests).
func (g *GPUHasher) lastPayloadUpload() (uint64, error) {
	g.mutex.Lock()
	defer g.mutex.Unlock()
	var n C.uint32_t
	if rc := C.msha_shard_count(g.ctx, &n); rc != C.MSHA_OK {
		return 0, g.fail(rc)
	}
	total := uint64(0)
	for i := C.uint32_t(0); i < n; i++ {
		var st C.msha_shard_stats
		if rc := C.msha_get_shard_stats(g.ctx, i, &st); rc != C.MSHA_OK {
			return 0, g.fail(rc)
		}
		total += uint64(st.h2d_payload_bytes)
	}
	return total, nil
}

// ensure returns p's buffer resized to n bytes (grown in pinned memory on demand).
func (g *GPUHasher) ensure(p *pinnedBuf, n int) ([]byte, error) {
	if cap(p.buf) >= n {
		p.buf = p.buf[:n]
		return p.buf, nil
	}
	if p.base != nil {
		C.msha_pinned_free(g.ctx, p.base)
		p.base, p.buf = nil, nil
	}
	size := n + n/4 + 4096
	var ptr unsafe.Pointer
	if rc := C.msha_pinned_alloc(g.ctx, C.uint64_t(size), &ptr); rc != C.MSHA_OK {
		return nil, g.fail(rc)
	}
	p.base = ptr
	p.buf = (*[1 << 40]byte)(ptr)[:n:size]
	return p.buf, nil
}

// words returns p's buffer resized to n uint64 values (pinned, grown on demand).
func (g *GPUHasher) words(p *pinnedBuf, n int) ([]uint64, error) {
	b, err := g.ensure(p, 8*n)
	if err != nil {
		return nil, err
	}
	return (*[1 << 37]uint64)(unsafe.Pointer(&b[0]))[:n:n], nil
}

// digests hashes n messages in one msha_digest_batch call. size bounds the
// packed arena (every packed message's bytes plus up to 15 bytes of alignment);
// pack(i, dst) copies message i's bytes to dst and returns their count. alias
// (nil, or one entry per message) names, for a message whose bytes equal an
// earlier message's, that earlier message (else -1): it is not packed again but
// gets the same (off, len), so its payload crosses PCIe once and the library
// hashes it once (msha_digest_batch folds equal (off, len)). Messages are
// placed 16-byte aligned and the arena, offsets, lengths and digests all live in
// pinned memory, so the library DMAs them as they are (no staging copy) and
// plans the lanes on the GPU. Returns n fresh 32-byte digests.
func (g *GPUHasher) digests(n int, size int, pack func(i int, dst []byte) int, alias []int) ([][]byte, error) {
	g.mutex.Lock()
	defer g.mutex.Unlock()
	if g.ctx == nil {
		return nil, errors.New("libmirsha: GPUHasher is closed")
	}
	result := make([][]byte, n)
	if n == 0 {
		return result, nil
	}
	arena, err := g.ensure(&g.arena, size+64)
	if err != nil {
		return nil, err
	}
	out, err := g.ensure(&g.out, 32*n)
	if err != nil {
		return nil, err
	}
	off, err := g.words(&g.off, n)
	if err != nil {
		return nil, err
	}
	length, err := g.words(&g.length, n)
	if err != nil {
		return nil, err
	}
	pos := 0
	for i := 0; i < n; i++ {
		if alias != nil && alias[i] >= 0 {
			off[i], length[i] = off[alias[i]], length[alias[i]]
			continue
		}
		off[i] = uint64(pos)
		l := pack(i, arena[pos:])
		length[i] = uint64(l)
		pos = (pos + l + 15) &^ 15
	}
	rc := C.msha_digest_batch(g.ctx,
		(*C.uint8_t)(unsafe.Pointer(&arena[0])), C.uint64_t(pos),
		(*C.uint64_t)(unsafe.Pointer(&off[0])), (*C.uint64_t)(unsafe.Pointer(&length[0])),
		C.uint64_t(n), (*C.uint8_t)(unsafe.Pointer(&out[0])))
	if rc != C.MSHA_OK {
		return nil, g.fail(rc)
	}
	digests := make([]byte, 32*n) // one allocation; each digest a capacity-capped slice of it
	copy(digests, out)
	for i := range result {
		result[i] = digests[32*i : 32*i+32 : 32*i+32]
	}
	return result, nil
}

// partsLen is the length of the concatenation of parts.
func partsLen(parts [][]byte) int {
	n := 0
	for _, p := range parts {
		n += len(p)
	}
	return n
}

// partsEqual reports whether two part lists concatenate to the same bytes
// (their part boundaries may differ).
func partsEqual(a, b [][]byte) bool {
	var x, y []byte
	for {
		for len(x) == 0 && len(a) > 0 {
			x, a = a[0], a[1:]
		}
		for len(y) == 0 && len(b) > 0 {
			y, b = b[0], b[1:]
		}
		if len(x) == 0 || len(y) == 0 {
			return len(x) == 0 && len(y) == 0
		}
		k := len(x)
		if len(y) < k {
			k = len(y)
		}
		if string(x[:k]) != string(y[:k]) {
			return false
		}
		x, y = x[k:], y[k:]
	}
}

// sameParts reports, in O(parts) and without reading payload bytes, whether
// two part lists hold the same bytes by construction: part for part, either the
// same slice (pointer and length: a message's own value and digest slices,
// stateless.go:330,338,345) or, for the short fresh slices the encoding makes
// (the BE64 fields, proposer.go:16-20), equal bytes. false means "not shown
// equal", not "different": the caller then compares bytes (partsEqual).
func sameParts(a, b [][]byte) bool {
	if len(a) != len(b) {
		return false
	}
	for k := range a {
		x, y := a[k], b[k]
		switch {
		case len(x) != len(y):
			return false
		case len(x) == 0:
		case len(x) <= 8:
			if string(x) != string(y) {
				return false
			}
		case &x[0] != &y[0]:
			return false
		}
	}
	return true
}

// epochChangeAliases finds the EpochChange hash actions whose payload an
// earlier action of the list already carries. A node hashes every origin's
// EpochChange once per ack (epoch_target.go:486-528, epoch_tracker.go:349-350):
// N^2 requests over N distinct payloads per epoch change. In the testengine
// the acks hold the originator's *msgs.EpochChange by pointer (recorder.go:39-47),
// so a pointer seen before is the same payload; acks deserialized from the
// network hold equal copies, found by comparing the bytes of earlier payloads
// from the same origin node with the same length (a byzantine copy that differs
// is packed and hashed on its own). A pointer hit aliases only when the two
// Data lists are shown equal -- part for part the same slices, or the same
// bytes (sameParts, else partsEqual) -- since the contract is SHA-256(Data),
// whatever message the Data was built from (batch_tracker.go:192-195: a wrong
// digest is a divergence). alias[i] = that earlier action, or -1.
func epochChangeAliases(reqs []*state.ActionHashRequest) (alias []int, size int) {
	type contentKey struct {
		origin uint64
		length int
	}
	alias = make([]int, len(reqs))
	var byPtr map[*msgs.EpochChange]int
	var byContent map[contentKey][]int
	for i, r := range reqs {
		alias[i] = -1
		l := partsLen(r.Data)
		if t, ok := r.Origin.GetType().(*state.HashOrigin_EpochChange_); ok && t.EpochChange != nil {
			ec := t.EpochChange
			if byPtr == nil {
				byPtr = map[*msgs.EpochChange]int{}
				byContent = map[contentKey][]int{}
			}
			// a pointer seen before names the same payload only if the Data built
			// from it is the same (the drop-in's contract is SHA-256(Data)): the
			// same slices in O(parts), else byte for byte
			if j, seen := byPtr[ec.EpochChange]; seen && ec.EpochChange != nil && partsLen(reqs[j].Data) == l &&
				(sameParts(reqs[j].Data, r.Data) || partsEqual(reqs[j].Data, r.Data)) {
				alias[i] = j
				continue
			}
			k := contentKey{ec.Origin, l}
			for _, j := range byContent[k] {
				if partsEqual(reqs[j].Data, r.Data) {
					alias[i] = j
					break
				}
			}
			if ec.EpochChange != nil {
				if alias[i] >= 0 {
					byPtr[ec.EpochChange] = alias[i]
				} else {
					byPtr[ec.EpochChange] = i
				}
			}
			if alias[i] >= 0 {
				continue
			}
			byContent[k] = append(byContent[k], i)
		}
		size += l + 15
	}
	return alias, size
}

// ProcessHashActionsGPU is a drop-in for ProcessHashActions (serial.go:180-198):
// one HashResult per action, in input order, Digest = SHA-256 of the action's
// Data parts concatenated (h.Write appends; zero parts hash the empty string),
// Origin the same pointer as the action's; a non-hash action fails the whole
// list with the reference's error text. One libmirsha call per ActionList; an
// EpochChange payload the list already carries is packed once and shared
// (epochChangeAliases).
func ProcessHashActionsGPU(g *GPUHasher, actions *statemachine.ActionList) (*statemachine.EventList, error) {
	reqs := make([]*state.ActionHashRequest, 0, actions.Len())
	iter := actions.Iterator()
	for action := iter.Next(); action != nil; action = iter.Next() {
		switch t := action.Type.(type) {
		case *state.Action_Hash:
			reqs = append(reqs, t.Hash)
		default:
			return nil, errors.Errorf("unexpected type for Hash action: %T", action.Type)
		}
	}

	alias, size := epochChangeAliases(reqs)
	digests, err := g.digests(len(reqs), size, func(i int, dst []byte) int {
		n := 0
		for _, data := range reqs[i].Data {
			n += copy(dst[n:], data)
		}
		return n
	}, alias)
	if err != nil {
		return nil, err
	}

	events := &statemachine.EventList{}
	for i, r := range reqs {
		events.HashResult(digests[i], r.Origin)
	}
	return events, nil
}

// RequestDigests returns SHA-256(data) for every request (clients.go:190-192),
// computed in one libmirsha call.
func (g *GPUHasher) RequestDigests(reqs []ProposedRequest) ([][]byte, error) {
	size := 0
	for _, r := range reqs {
		size += len(r.Data) + 15
	}
	return g.digests(len(reqs), size, func(i int, dst []byte) int {
		return copy(dst, reqs[i].Data)
	}, nil)
}
