// Reference header name (include/gmm.h) mapped onto the MI355X host API.
#pragma once
#include "vol_renderer.h"
