// Reference header name (include/integrator.h) mapped onto the MI355X host API.
#pragma once
#include "vol_renderer.h"
