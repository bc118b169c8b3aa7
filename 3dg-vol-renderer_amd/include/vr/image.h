// Reference header name (include/image.h) mapped onto the MI355X host API.
#pragma once
#include "vol_renderer.h"
