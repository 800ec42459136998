// Internal declarations shared by the host-side translation units.
#pragma once
#include <string>

#include "nori_hip.h"

namespace nh {
void set_host_error(const std::string &msg);
}
