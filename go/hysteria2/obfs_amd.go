//go:build linux && sqobfs

// The MI355X build of Hysteria2's Salamander decorator: replaces
// hysteria2/salamander.go (which the maintainer tags `//go:build !sqobfs`)
// with the same exported names and signatures, so the construction sites
// (hysteria2/client.go:133-135, hysteria2/service.go:118-120) compile
// unchanged.  Byte work: libsqobfs on the GPU, batched (go/sqobfs).
// Uncompiled here (no Go toolchain in this image); the C call sequence is
// replayed by tests/cpp/test_cgo_sequence.c.
package hysteria2

import (
	"net"

	"github.com/sagernet/sing-quic/internal/sqobfs"
	"github.com/sagernet/sing/common/buf"
	"github.com/sagernet/sing/common/bufio"
	M "github.com/sagernet/sing/common/metadata"
	N "github.com/sagernet/sing/common/network"
)

const salamanderSaltLen = 8 // salamander.go:15

const ObfsTypeSalamander = "salamander" // salamander.go:17

// SalamanderPacketConn: salamander.go:19-22, the byte work on the GPU.
type SalamanderPacketConn = sqobfs.Conn

// NewSalamanderConn keeps salamander.go:24's signature.  There is no CPU
// fallback: without a GPU it panics, as a misconfigured build should.
func NewSalamanderConn(conn net.PacketConn, password []byte) net.PacketConn {
	c, err := sqobfs.NewConn(conn, sqobfs.Salamander, password, sqobfs.Options{})
	if err != nil {
		panic("sqobfs: " + err.Error())
	}
	if writer, isVectorised := bufio.CreateVectorisedPacketWriter(conn); isVectorised {
		return &VectorisedSalamanderPacketConn{Conn: c, writer: writer}
	}
	return c
}

// VectorisedSalamanderPacketConn: salamander.go:76-109.
type VectorisedSalamanderPacketConn struct {
	*sqobfs.Conn
	writer N.VectorisedPacketWriter
}

// WriteVectorisedPacket obfuscates the concatenation of buffers under one
// key: the intent of salamander.go:95-109 (its line 104 mis-indexes any
// buffer after the first; XPlus's xplus.go:100-118 does it right).
func (v *VectorisedSalamanderPacketConn) WriteVectorisedPacket(buffers []*buf.Buffer,
	destination M.Socksaddr) error {
	defer buf.ReleaseMulti(buffers)
	n := buf.LenMulti(buffers)
	p := make([]byte, 0, n)
	for _, b := range buffers {
		p = append(p, b.Bytes()...)
	}
	_, err := v.Conn.WriteTo(p, destination.UDPAddr())
	return err
}
