//go:build linux && sqobfs

// The MI355X build of Hysteria v1's XPlus decorator: replaces
// hysteria/xplus.go (tagged `//go:build !sqobfs` by the maintainer) with the
// same exported names and signatures (construction sites
// hysteria/client.go:185-187, hysteria/service.go:130-132).  Uncompiled
// here (no Go toolchain in this image).
package hysteria

import (
	"net"

	"github.com/sagernet/sing-quic/internal/sqobfs"
	"github.com/sagernet/sing/common/buf"
	"github.com/sagernet/sing/common/bufio"
	M "github.com/sagernet/sing/common/metadata"
)

const xplusSaltLen = 16 // xplus.go:17

// XPlusPacketConn: xplus.go:39-44.  Its salts come from the context's
// ChaCha20 generator (on the GPU, or the same stream on the CPU path) instead
// of a mutex-guarded math/rand (xplus.go:26,34,67-69).
type XPlusPacketConn = sqobfs.Conn

// NewXPlusPacketConn keeps xplus.go:19's signature and, like it, does not
// fail for want of a GPU (the CPU path then does every batch); only a process
// out of memory or threads panics here.
func NewXPlusPacketConn(conn net.PacketConn, key []byte) net.PacketConn {
	c, err := sqobfs.NewConn(conn, sqobfs.XPlus, key, sqobfs.Options{})
	if err != nil {
		panic("sqobfs: " + err.Error())
	}
	if _, isVectorised := bufio.CreateVectorisedPacketWriter(conn); isVectorised {
		return &VectorisedXPlusConn{Conn: c} // the engine sends: no inner writer kept
	}
	return c
}

// VectorisedXPlusConn: xplus.go:81-118 (one running keystream over the
// buffers, as :108-115).  WriteTo copies p (xplus.go:94-96 XORs it in place).
type VectorisedXPlusConn struct {
	*sqobfs.Conn
}

func (v *VectorisedXPlusConn) WriteVectorisedPacket(buffers []*buf.Buffer,
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
