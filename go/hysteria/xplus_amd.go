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
	N "github.com/sagernet/sing/common/network"
)

const xplusSaltLen = 16 // xplus.go:17

// XPlusPacketConn: xplus.go:39-44.  Its salts come from the GPU's ChaCha20
// generator instead of a mutex-guarded math/rand (xplus.go:26,34,67-69).
type XPlusPacketConn = sqobfs.Conn

// NewXPlusPacketConn keeps xplus.go:19's signature.
func NewXPlusPacketConn(conn net.PacketConn, key []byte) net.PacketConn {
	c, err := sqobfs.NewConn(conn, sqobfs.XPlus, key, sqobfs.Options{})
	if err != nil {
		panic("sqobfs: " + err.Error())
	}
	if writer, isVectorised := bufio.CreateVectorisedPacketWriter(conn); isVectorised {
		return &VectorisedXPlusConn{Conn: c, writer: writer}
	}
	return c
}

// VectorisedXPlusConn: xplus.go:81-118 (one running keystream over the
// buffers, as :108-115).
type VectorisedXPlusConn struct {
	*sqobfs.Conn
	writer N.VectorisedPacketWriter
}

func (v *VectorisedXPlusConn) WriteVectorisedPacket(buffers []*buf.Buffer,
	destination M.Socksaddr) error {
	defer buf.ReleaseMulti(buffers)
	p := make([]byte, 0, buf.LenMulti(buffers))
	for _, b := range buffers {
		p = append(p, b.Bytes()...)
	}
	_, err := v.Conn.WriteTo(p, destination.UDPAddr())
	return err
}
