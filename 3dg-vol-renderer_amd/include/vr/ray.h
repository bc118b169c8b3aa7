// Reference header name (include/ray.h) mapped onto the MI355X host API.
#pragma once
#include "vol_renderer.h"
