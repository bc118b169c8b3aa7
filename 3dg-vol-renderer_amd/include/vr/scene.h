// Reference header name (include/scene.h) mapped onto the MI355X host API.
#pragma once
#include "vol_renderer.h"
