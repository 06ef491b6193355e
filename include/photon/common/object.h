/*
 * photon/common/object.h -- the one type of PhotonLibOS's common/object.h:19-23
 * that the vDMA interface (photon/net/vdma.h) derives from. In a Photon build
 * Photon's own header (same path) is used instead; the class is identical.
 */
#pragma once

namespace photon {

class Object {
public:
    virtual ~Object() {}
};

}  // namespace photon
