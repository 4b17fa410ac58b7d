//go:build linux && sqobfs

// The MI355X build of Hysteria2's Salamander decorator: replaces
// hysteria2/salamander.go (which the maintainer tags `//go:build !sqobfs`)
// with the same exported names and signatures, so the construction sites
// (hysteria2/client.go:133-135, hysteria2/service.go:118-120) compile
// unchanged.  Byte work: libsqobfs on the GPU, batched (go/sqobfs), or on its
// CPU path for small batches and when there is no GPU.
// Uncompiled here (no Go toolchain in this image); the engine under
// sqobfs.Conn is tested natively by tests/cpp/test_pconn.c.
package hysteria2

import (
	"net"

	"github.com/sagernet/sing-quic/internal/sqobfs"
	"github.com/sagernet/sing/common/buf"
	"github.com/sagernet/sing/common/bufio"
	M "github.com/sagernet/sing/common/metadata"
)

const salamanderSaltLen = 8 // salamander.go:15

const ObfsTypeSalamander = "salamander" // salamander.go:17

// SalamanderPacketConn: salamander.go:19-22, the byte work on the GPU.
type SalamanderPacketConn = sqobfs.Conn

// NewSalamanderConn keeps salamander.go:24's signature, and like it cannot
// fail for want of a device: without a usable GPU the Conn runs every batch
// on the library's CPU path (sqobfs.NewConn).  Only a process out of memory
// or threads panics here, as the Go runtime itself would.
func NewSalamanderConn(conn net.PacketConn, password []byte) net.PacketConn {
	c, err := sqobfs.NewConn(conn, sqobfs.Salamander, password, sqobfs.Options{})
	if err != nil {
		panic("sqobfs: " + err.Error())
	}
	if _, isVectorised := bufio.CreateVectorisedPacketWriter(conn); isVectorised {
		// the reference keeps the inner vectorised writer (salamander.go:25-
		// 33); here the engine sends, so only the method set is kept
		return &VectorisedSalamanderPacketConn{Conn: c}
	}
	return c
}

// VectorisedSalamanderPacketConn: salamander.go:76-109.  Its WriteTo is
// sqobfs.Conn's, which copies p instead of XORing it in place
// (salamander.go:85-87 mutates the caller's p; callers do not read it back).
type VectorisedSalamanderPacketConn struct {
	*sqobfs.Conn
}

// WriteVectorisedPacket obfuscates the concatenation of buffers under one
// key: the intent of salamander.go:95-109 (its line 104 mis-indexes any
// buffer after the first; XPlus's xplus.go:100-118 does it right).  The
// buffers are gathered into a pooled buffer; WriteTo copies it into the
// transmit batch.
func (v *VectorisedSalamanderPacketConn) WriteVectorisedPacket(buffers []*buf.Buffer,
	destination M.Socksaddr) error {
	defer buf.ReleaseMulti(buffers)
	p := buf.NewSize(buf.LenMulti(buffers))
	defer p.Release()
	for _, b := range buffers {
		_, _ = p.Write(b.Bytes())
	}
	_, err := v.Conn.WriteTo(p.Bytes(), destination.UDPAddr())
	return err
}
