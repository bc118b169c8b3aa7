// Reference header name (include/test_integrators.h) mapped onto the MI355X host API.
#pragma once
#include "vol_renderer.h"
