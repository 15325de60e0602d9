from .resource import (RESOURCE_NAME_PREFIX, STRATEGY_MIXED, STRATEGY_NONE, STRATEGY_SINGLE, Resource,  # noqa: F401
                       ResourceName, new_resource)
from .resources import new_resources, profile_name  # noqa: F401
