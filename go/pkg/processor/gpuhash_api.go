// The part of the GPU-batched hash API that both builds share: it has no cgo
// and compiles with or without the mirsha build tag. GPUHasher, NewGPUHasher,
// Close, RequestDigests and ProcessHashActionsGPU come from gpuhash.go (tag
// mirsha: libmirsha over cgo) or gpuhash_stub.go (no tag: every call reports
// that the library is not built in).
//
// Go 1.15 compatible (go.mod:3).
package processor

import (
	"github.com/pkg/errors"

	"github.com/hyperledger-labs/mirbft/pkg/statemachine"
)

// ProposedRequest is one request of a ProposeBatch call.
type ProposedRequest struct {
	ReqNo uint64
	Data  []byte
}

// ProposeBatch is Client.Propose (clients.go:189-276) for several requests of
// this client. Their digests come from one libmirsha call; then each request
// runs Propose's bookkeeping (proposeDigest) in order, so the request store,
// the allocation state and the returned events are exactly those of calling
// Propose once per request in the same order. The result is the concatenation
// of the per-request event lists; the first error stops the batch and is
// returned with the events of the requests before it.
func (c *Client) ProposeBatch(g *GPUHasher, reqs []ProposedRequest) (*statemachine.EventList, error) {
	digests, err := g.RequestDigests(reqs)
	if err != nil {
		return nil, errors.WithMessage(err, "could not hash requests")
	}
	events := &statemachine.EventList{}
	for i, r := range reqs {
		el, err := c.proposeDigest(r.ReqNo, r.Data, digests[i])
		if err != nil {
			return events, err
		}
		events.PushBackList(el)
	}
	return events, nil
}
