// render/Scene.h — the reference's scene model (libs/render/include/render/Scene.h:13-227), the part
// the App and the integrator use: SceneNode {id, name, type, position}, SphereObject {radius} and the
// Scene registry with its change flag, with the reference's member names, container types and
// change-flag semantics (CreateNode does not re-flag, Scene.h:207-215).
//
// Positions are glm::vec3 when glm is on the include path (the reference's build: App.cpp:104 calls
// SetPosition(glm::vec3(...))); this image has no glm, so then they are a three-float render::Vec3.
// The backend (HIPPathTracer.cpp) reads GetPosition() through .x/.y/.z only, so it compiles against
// either this header or the reference's own (tests/test_cpp_interface.py checks the latter).
// Transforms/quaternions, unused by the integrator, are omitted.
#pragma once

#include <algorithm>
#include <cstdint>
#include <memory>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#if __has_include(<glm/glm.hpp>)
#include <glm/glm.hpp>
namespace render
{
	using Vec3 = glm::vec3;
}
#else
namespace render
{
	struct Vec3
	{
		float x = 0.0f, y = 0.0f, z = 0.0f;
		Vec3() = default;
		explicit Vec3(float s) : x(s), y(s), z(s) {}
		Vec3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
	};
}
#endif

namespace render
{
	using NodeID = uint32_t;

	enum class NodeType
	{
		SCENE_ROOT,
		SPHERE_OBJECT,
		MATERIAL,
		GROUP
	};

	class SceneNode
	{
	protected:
		static inline NodeID s_nextID = 0;  // Scene.cpp:8
		NodeID m_id;
		std::string m_name;
		NodeType m_type;
		Vec3 m_position{0.0f, 0.0f, 0.0f};  // Transform::position (Scene.h:24)

	public:
		SceneNode(NodeType type, const std::string &name = "Node") : m_id(s_nextID++), m_name(name), m_type(type) {}
		virtual ~SceneNode() = default;

		NodeID GetID() const { return m_id; }
		const std::string &GetName() const { return m_name; }
		void SetName(const std::string &name) { m_name = name; }
		NodeType GetType() const { return m_type; }

		void SetPosition(const Vec3 &position) { m_position = position; }
		Vec3 GetPosition() const { return m_position; }
	};

	class SphereObject : public SceneNode
	{
	private:
		float m_radius = 1.0f;

	public:
		SphereObject(const std::string &name = "Sphere") : SceneNode(NodeType::SPHERE_OBJECT, name) {}
		float GetRadius() const { return m_radius; }
		void SetRadius(float radius) { m_radius = radius; }
	};

	class Scene
	{
	private:
		std::unique_ptr<SceneNode> m_rootNode;
		// keyed by NodeID in an unordered_map as in the reference (Scene.h:140): the integrator's
		// primitive order is this map's iteration order, as the reference's Embree geomIDs are
		std::unordered_map<NodeID, SceneNode *> m_nodeRegistry;
		std::vector<std::unique_ptr<SceneNode>> m_nodes;
		bool m_has_changes = true;

	public:
		Scene() : m_rootNode(std::make_unique<SceneNode>(NodeType::SCENE_ROOT, "Root")) {}

		SceneNode *GetRootNode() const { return m_rootNode.get(); }
		const std::unordered_map<NodeID, SceneNode *> &GetAllNodes() const { return m_nodeRegistry; }

		template <typename T, typename... Args>
		T *CreateNode(Args &&...args)
		{
			static_assert(std::is_base_of<SceneNode, T>::value, "T must be derived from SceneNode");
			auto node = std::make_unique<T>(std::forward<Args>(args)...);
			T *ptr = node.get();
			m_nodeRegistry[ptr->GetID()] = ptr;
			m_nodes.push_back(std::move(node));
			return ptr;
		}

		bool DeleteNode(NodeID id)
		{
			auto it = m_nodeRegistry.find(id);
			if (it == m_nodeRegistry.end())
				return false;
			SceneNode *node = it->second;
			m_nodeRegistry.erase(it);
			auto owned = std::find_if(m_nodes.begin(), m_nodes.end(),
									  [node](const std::unique_ptr<SceneNode> &p) { return p.get() == node; });
			if (owned != m_nodes.end())
				m_nodes.erase(owned);
			return true;
		}

		SceneNode *FindNode(NodeID id)
		{
			auto it = m_nodeRegistry.find(id);
			return it != m_nodeRegistry.end() ? it->second : nullptr;
		}

		SceneNode *FindNode(const std::string &name)
		{
			for (const auto &[id, node] : m_nodeRegistry)
				if (node->GetName() == name)
					return node;
			return nullptr;
		}

		bool hasChanges() const { return m_has_changes; }
		void markChangesProcessed() { m_has_changes = false; }
	};
} // namespace render
